#!/bin/bash
# Round 6m: tile-family next-tile prefetch (QDC_TILE_PF 0 / 1) x reduction grid (QDC_RED_CAP
# 2048 / 4096) on single-gate cells; k_diag_q at its new defaults (16 in flight, 4096 blocks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6m
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_primitives.py -x -q --timeout 200 \
  --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
for rep in 1 2; do
for cfg in "0 2048" "1 2048" "0 4096" "1 4096"; do
  set -- $cfg
  QDC_TILE_PF=$1 QDC_RED_CAP=$2 timeout -k 10 300 python -u tools/r5/micro_subset.py --q1 0,12,20,24,27 \
    --q2 0:1,5:20,26:27,14:13,1:2,3:9,27:0 > "$OUT/micro_pf$1_r$2_$rep.log" 2>&1 || exit $?
  echo "pf $1 redcap $2 rep $rep done"
done
done
tail -2 "$OUT/tests.log"
