#!/bin/bash
# Tile-far default (reverse ops): its parity test, the micro sweep, then the LCMIN A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2o; mkdir -p $OUT; export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_primitives.py -x -v -s --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
grep -E "passed|failed" $OUT/tests.log | tail -1
echo "== micro $(date +%T)"
timeout -k 10 400 python -u bench.py --micro > $OUT/micro.log 2>&1 || { tail -20 $OUT/micro.log; exit 1; }
python3 tools/micro_table.py $OUT/micro.log > $OUT/micro_table.txt
echo "== lc $(date +%T)"
TAG=r2o_lc bash tools/lc_ab.sh
