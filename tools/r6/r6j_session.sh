#!/bin/bash
# Round 6j: static share of the register-resident passes' dynamic tail (QDC_DYN, % of the fair
# share run block-contiguously; the rest comes in increasing order from per-XCD pool counters):
# same-box A/B of the bench step, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6j
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do for d in 35 0 15 60; do
  QDC_DYN=$d timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gate-sample \
    > "$OUT/bench_dyn$d.json" 2> "$OUT/bench_dyn$d.err" || exit $?
  python3 -c "
import json; s=open('$OUT/bench_dyn$d.json').read(); L=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
k=L['kernels']; print('dyn $d', L['value'], L['ms_per_step'], 'rev', k['fused_reverse']['avg_ms'], 'apply', k['fused_apply']['avg_ms'])" | tee -a "$OUT/ab.txt"
done; done
