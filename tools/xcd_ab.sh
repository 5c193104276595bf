#!/bin/bash
# XCD-aware block order of the direct single-gate launches: parity with it on, then the micro
# sweep with it off and on (same box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-xcd}; mkdir -p $OUT; export TMPDIR=/tmp
QDC_XCD_MAP=${XCD_TEST:-1} timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_golden.py tests/test_gpu_layout.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_xcd1.log 2>&1 || { tail -30 $OUT/tests_xcd1.log; exit 1; }
tail -1 $OUT/tests_xcd1.log
for v in ${XCD_VALS:-0 1}; do
  QDC_XCD_MAP=$v timeout -k 10 400 python -u bench.py --micro > $OUT/micro_xcd$v.log 2>&1 || { tail -20 $OUT/micro_xcd$v.log; exit 1; }
  python3 tools/micro_table.py $OUT/micro_xcd$v.log > $OUT/micro_table_xcd$v.txt
done
echo done
