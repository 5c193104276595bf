#!/bin/bash
# Round 6s (after 6r): the state-pair interleave granule (QDC_STATE_ILV_BITS 12 = 64 KiB blocks, the
# default; 14; 16) on the single-gate reverse cells and on a short C2 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6s
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1; do
for b in 10 11 13; do
  QDC_STATE_ILV_BITS=$b timeout -k 10 300 python -u tools/r5/micro_subset.py --q1 0,20 \
    --q2 14:13,26:27,5:20,0:1 > "$OUT/micro_ilv${b}_${rep}.log" 2>&1 || exit $?
  echo "ilv $b $(grep -E 'reverse_q' "$OUT/micro_ilv${b}_${rep}.log" | awk '{for(i=1;i<=NF;i++) if($i ~ /%$/) p=$i; print $2,$3,p}' | tr '\n' ' ')" | tee -a "$OUT/ilv_ab.txt"
  QDC_STATE_ILV_BITS=$b timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-gate-sample \
    > "$OUT/bench_ilv${b}_${rep}.json" 2> "$OUT/bench_ilv${b}_${rep}.err" || exit $?
  python3 -c "
import json; s=open('$OUT/bench_ilv${b}_${rep}.json').read(); L=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
print('ilv $b bench', L['value'], L['ms_per_step'], 'rev', L['kernels']['fused_reverse']['avg_ms'], 'apply', L['kernels']['fused_apply']['avg_ms'])" | tee -a "$OUT/ilv_ab.txt"
done
done
