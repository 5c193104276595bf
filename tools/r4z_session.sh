#!/bin/bash
# Dense-gate LDS tiles: pipelined variants (QDC_QKL_VAR) A/B with an experimental library in
# qkx/, parity of each variant first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4z
mkdir -p "$OUT"
export QDC_LIB_DIR=$PWD/qkx
for v in 1 2; do
  QDC_QKL_VAR=$v timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dense.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests_$v.log" 2>&1 || { tail -30 "$OUT/tests_$v.log"; exit 1; }
  tail -1 "$OUT/tests_$v.log"
done
for rep in 1 2; do
for v in 0 1 2; do
  echo "QDC_QKL_VAR=$v" >> "$OUT/pos.log"
  QDC_QKL_VAR=$v timeout -k 10 240 python3 tools/qk_pos_probe.py >> "$OUT/pos.log" 2>&1 || exit $?
done
done
grep -E "VAR|bench" "$OUT/pos.log"
