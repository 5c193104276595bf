#!/bin/bash
# A single-gate knob (KNOB, values VALS): parity of the single-gate tests with TESTVAL, then the
# micro sweep per value (same box).  Every GPU step time-boxed; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-knob}; mkdir -p $OUT; export TMPDIR=/tmp
env $KNOB=$TESTVAL timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_golden.py tests/test_gpu_layout.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in $VALS; do
  env $KNOB=$v timeout -k 10 400 python -u bench.py --micro > $OUT/micro_$v.log 2>&1 || { tail -20 $OUT/micro_$v.log; exit 1; }
  python3 tools/micro_table.py $OUT/micro_$v.log > $OUT/micro_table_$v.txt
done
echo done
