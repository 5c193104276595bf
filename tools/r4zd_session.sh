#!/bin/bash
# Dense-gate LDS tiles for every placement (QDC_QK_LDS=-1) against the default, experimental
# library in qkx/ (built with "lds_min != 0" in apply_qk, so that -1 stages every gate; the
# committed library treats -1 as 0): parity, then bench.py's placements and the placement probe, two repeats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4zd
mkdir -p "$OUT"
export QDC_LIB_DIR=$PWD/qkx
QDC_QK_LDS=-1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dense.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do
for v in default -1; do
  echo "QDC_QK_LDS=$v" >> "$OUT/pos.log"
  if [ $v = default ]; then timeout -k 10 240 python3 tools/qk_pos_probe.py >> "$OUT/pos.log" 2>&1 || exit $?
  else QDC_QK_LDS=$v timeout -k 10 240 python3 tools/qk_pos_probe.py >> "$OUT/pos.log" 2>&1 || exit $?; fi
done
done
cat "$OUT/pos.log"
