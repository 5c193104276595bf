#!/bin/bash
# Round 6v: the whole single-gate sweep (every q1 position, the 8 q2 pairs) with the default
# LANE family, with its block-wide variant off (QDC_LANE_BLK=0) and with streaming ops on the
# tile family (QDC_LANE=0), interleaved, two repeats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6v
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in base QDC_LANE_BLK=0 QDC_LANE=0; do
  env $( [ "$cfg" = base ] || echo "$cfg" ) timeout -k 10 400 python -u tools/r5/micro_subset.py \
    --q1 0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25,26,27 \
    --q2 0:1,1:0,5:20,26:27,27:0,1:2,3:9,14:13 > "$OUT/micro_${cfg}_${rep}.log" 2>&1 || exit $?
  echo "$cfg rep $rep done"
done
done
