#!/bin/bash
# Round 6h: same-box A/B of the final library against the r6b library (commit 334eac6, built
# into abtree/b2 with its own headers and prebuilt kernels): is the slower r6d-r6g boxes'
# headline the box or the round's last changes?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6h
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gate-sample \
    > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || exit $?
  python3 -c "
import json; s=open('$OUT/bench_$tag.json').read(); L=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
k=L['kernels']; print('$tag', L['value'], L['ms_per_step'], 'rev', k['fused_reverse']['avg_ms'], 'apply', k['fused_apply']['avg_ms'], 'dens', k['fused_density']['avg_ms'], 'compiled', L['ranks'][0]['kernels_compiled'])" | tee -a "$OUT/ab.txt"
}
for i in 1 2; do
  run final QDC_BENCH_UNPROFILED_STEPS=10
  run r6b QDC_LIB_DIR=$PWD/abtree/b2/pkg/lib QDC_BENCH_UNPROFILED_STEPS=10
done
