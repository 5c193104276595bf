#!/bin/bash
# Round 6w: the address-map exceptions of the one-state application (QDC_LANE_TILE_BITS,
# QDC_LANE_NOBLK_BITS) against the round-6v defaults (both masks 0), and the single-gate tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6w
mkdir -p "$OUT"
export TMPDIR=/tmp
QDC_FUSE=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_primitives.py -x -q --timeout 300 \
  --timeout-method thread -k "not large_state" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
for rep in 1 2; do
for cfg in new old; do
  envs=""; [ $cfg = old ] && envs="QDC_LANE_TILE_BITS=0 QDC_LANE_NOBLK_BITS=0"
  env $envs timeout -k 10 300 python -u tools/r5/micro_subset.py --q1 11,12,13,19,20,21,23,24,25 \
    --q2 5:20,3:9,14:13 > "$OUT/micro_${cfg}_${rep}.log" 2>&1 || exit $?
  echo "$cfg $(grep -E 'apply_q' "$OUT/micro_${cfg}_${rep}.log" | grep -v diag | awk '{for(i=1;i<=NF;i++) if($i ~ /%$/) p=$i; print $2,p}' | tr '\n' ' ')" | tee -a "$OUT/ab.txt"
done
done
tail -2 "$OUT/tests.log"
