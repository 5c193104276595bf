#!/bin/bash
# Round 6o: the two far-far reverse_q2 cells under existing knobs (direct rows for far reverse
# targets, 2^10-chunk two-state tiles, XCD order of reducing launches, LANE reverse).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6o
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "base" "QDC_TILE_FAR=2" "QDC_TILE2_WIDE=1" "QDC_XCD_MAP=3" "QDC_LANE=3"; do
  env $( [ "$cfg" = base ] || echo "$cfg" ) timeout -k 10 300 python -u tools/r5/micro_subset.py \
    --q2 14:13,26:27,5:20,27:0 > "$OUT/micro_${cfg}_$rep.log" 2>&1 || exit $?
  echo "$cfg $(grep -E 'reverse_q2 ' "$OUT/micro_${cfg}_$rep.log" | awk '{for(i=1;i<=NF;i++) if($i ~ /%$/) p=$i; print $2,p}' | tr '\n' ' ')" | tee -a "$OUT/far_ab.txt"
done
done
