#!/bin/bash
# Round 6n: the single-gate defaults of round 6 (k_diag_q 16 in flight / 4096 blocks, reverse
# launches on 4096 blocks, tile prefetch without row bits): single-gate parity tests, then the
# subset of cells against the round-5 defaults (QDC_DIAG_Q=0 QDC_DIAG_RU=8 QDC_REV_RED=2048
# QDC_TILE_PF=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6n
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_primitives.py tests/test_gpu_golden.py \
  -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
for rep in 1 2; do
  timeout -k 10 300 python -u tools/r5/micro_subset.py --q1 0,12,20,24,27 \
    --q2 0:1,5:20,26:27,14:13,1:2,3:9,27:0 > "$OUT/micro_new_$rep.log" 2>&1 || exit $?
  QDC_DIAG_Q=0 QDC_DIAG_RU=8 QDC_REV_RED=2048 QDC_TILE_PF=0 timeout -k 10 300 python -u tools/r5/micro_subset.py \
    --q1 0,12,20,24,27 --q2 0:1,5:20,26:27,14:13,1:2,3:9,27:0 > "$OUT/micro_old_$rep.log" 2>&1 || exit $?
done
tail -2 "$OUT/tests.log"
