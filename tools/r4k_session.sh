#!/bin/bash
# Widest single-gate tiles (QDC_TILE{1,2}_WIDE=2): parity, then the weak cells per tile width
# and family.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4k}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_layout.py -x -v -s --timeout 200 --timeout-method thread -k far_target \
  > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed" "$OUT/tests.log" | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u tools/micro_tune.py --reps 2 --q1 1,3,20,22,24 --q2 5:20,26:27,14:13 --out "$OUT/micro_tune.json" \
  --cfgs "- QDC_TILE2_WIDE=2 QDC_TILE_FAR=3,QDC_TILE1_WIDE=2 QDC_TILE_FAR=3,QDC_TILE1_WIDE=2,QDC_TILE2_WIDE=2 QDC_TILE_FAR=3,QDC_TILE1_WIDE=2,QDC_XCD_MAP=0" \
  > "$OUT/micro_tune.log" 2>&1 || exit $?
grep -E "apply|reverse" "$OUT/micro_tune.log"
