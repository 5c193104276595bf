#!/bin/bash
# Round 5n: the weak single-gate cells (far rows at DRAM-unfriendly distances) under block order
# and block-wide lane variants; reductions under XCD order and a larger grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5n
mkdir -p "$OUT"
export TMPDIR=/tmp
S="--q1 12,18,19,20,21,23,24,25 --q2 5:20,26:27,14:13,3:9"
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u tools/r5/micro_subset.py $S > "$OUT/micro_$tag.log" 2>&1 || { tail -20 "$OUT/micro_$tag.log"; exit 1; }
}
run blk1 QDC_LANE_BLK=1
run blk0 QDC_LANE_BLK=0
run blk1_x0 QDC_LANE_BLK=1 QDC_XCD_MAP=0
run blk0_x0 QDC_LANE_BLK=0 QDC_XCD_MAP=0
run blk0_x3 QDC_LANE_BLK=0 QDC_XCD_MAP=3
run blk0_rc4k QDC_LANE_BLK=0 QDC_RED_CAP=4096
run blk1c QDC_LANE_BLK=1
