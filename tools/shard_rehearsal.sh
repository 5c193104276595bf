#!/bin/bash
# The sharded data path rehearsed on one GPU at the bench workload (C2, n = 28): unsharded
# (default and with the two features the sharded path lacks: permuting passes, interleaved
# state pair), G local shards on one stream, G shards on their own streams.  Per configuration
# one bench line (kernels, all-to-all copy time, the planner's remaps per step); every GPU step
# time-boxed, the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-shard}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -k 10 400 env "$@" python bench.py --steps ${STEPS_N:-2} --warmup 1 --no-cpu-baseline \
    --no-gate-sample ${BENCH_ARGS} > "$OUT/b_$tag.log" 2>&1 || { tail -5 "$OUT/b_$tag.log"; exit 1; }
  python3 - "$OUT/b_$tag.log" "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], d["value"], "gates/s", d["ms_per_step"], "ms/step remaps", d["config"]["remaps_per_step"],
      {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.005})
PY
}
run unsharded QDC_X=0
run unsharded_noperm_noilv QDC_RQ_PERM=0 QDC_STATE_ILV=0
for g in ${SHARDS:-2 4 8}; do
  BENCH_ARGS="$BENCH_ARGS --local-shards $g" run shards$g QDC_X=0
done
for g in ${STREAMS:-2 4}; do
  BENCH_ARGS="$BENCH_ARGS --local-streams $g" run streams$g QDC_X=0
done
