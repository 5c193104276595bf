#!/bin/bash
# Round 6i: same-box A/B of the profiler's event kind on the final library (QDC_EVENT_FENCE 0:
# timing-only, 1: default events) beside the r6b library, three rounds, with host phase times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6i
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  env "$@" QDC_BENCH_UNPROFILED_STEPS=10 timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 \
    --no-cpu-baseline --no-gate-sample > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || exit $?
  python3 -c "
import json; s=open('$OUT/bench_$tag.json').read(); L=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
k=L['kernels']; h=L['host_ms_per_step']
print('$tag', L['value'], L['ms_per_step'], 'unprof', L['unprofiled_ms_per_step'], 'rev', k['fused_reverse']['avg_ms'], 'apply', k['fused_apply']['avg_ms'],
      'host f', round(h['forward']['setup']+h['forward']['schedule']+h['forward']['build'],3), round(h['forward']['launch'],3),
      'b', round(h['backward']['setup']+h['backward']['schedule']+h['backward']['build'],3), round(h['backward']['launch'],3))" | tee -a "$OUT/ab.txt"
}
for i in 1 2 3; do
  run final_nofence$i QDC_EVENT_FENCE=0
  run final_fence$i QDC_EVENT_FENCE=1
  run r6b$i QDC_LIB_DIR=$PWD/abtree/b2/pkg/lib
done
