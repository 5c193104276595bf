#!/bin/bash
# Round 6u: the far one-state apply cells (q1 20 / 24, q2 (5,20)) under the LANE knobs: units in
# flight per wave of streaming launches (QDC_LANE_U second field 1 / 4 / 8), the block-wide
# variant off (QDC_LANE_BLK=0), and the tile family (QDC_LANE=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6u
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in base QDC_LANE_U=8,4,4 QDC_LANE_U=8,8,4 QDC_LANE_BLK=0 QDC_LANE_BLK=0,QDC_LANE_U=8,4,4 QDC_LANE=0; do
  envs=$( [ "$cfg" = base ] || echo "$cfg" | sed 's/,QDC/ QDC/g' )
  env $envs timeout -k 10 300 python -u tools/r5/micro_subset.py --q1 20,24,12,3 --q2 5:20,26:27 \
    > "$OUT/micro_${cfg}_${rep}.log" 2>&1 || exit $?
  echo "$cfg $(grep -E 'apply_q' "$OUT/micro_${cfg}_${rep}.log" | grep -v diag | awk '{for(i=1;i<=NF;i++) if($i ~ /%$/) p=$i; print $2,$3,p}' | tr '\n' ' ')" | tee -a "$OUT/lane_ab.txt"
done
done
