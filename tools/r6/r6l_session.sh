#!/bin/bash
# Round 6l: k_diag_q units in flight (QDC_DIAG_RU 4 / 8 / 16) and reduction grid (QDC_RED_CAP
# 1024 / 2048 / 4096) on the diagonal reverse cells.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6l
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
for cfg in "8 2048" "4 2048" "16 2048" "8 1024" "8 4096" "16 4096"; do
  set -- $cfg
  QDC_DIAG_RU=$1 QDC_RED_CAP=$2 timeout -k 10 300 python -u tools/r5/micro_subset.py \
    --q2 0:1,5:20,26:27,14:13 > "$OUT/micro_u$1_r$2.log" 2>&1 || exit $?
  echo "ru $1 redcap $2 $(grep -E 'reverse_q2_diag' "$OUT/micro_u$1_r$2.log" | awk '{for(i=1;i<=NF;i++) if($i ~ /%$/) p=$i; print $3,p}' | tr '\n' ' ')" | tee -a "$OUT/diag_ru_ab.txt"
done
done
