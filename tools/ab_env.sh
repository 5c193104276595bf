#!/bin/bash
# GPU A/B of runtime knobs on the C2 bench: optional parity subset first (TESTS, pytest
# args), then one short bench per configuration in CFGS (space separated; each a comma
# separated list of VAR=VALUE, "-" for the defaults), interleaved REPS times.  Every GPU step
# is time-boxed; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${REPS:-1}); do
  for cfg in ${CFGS:--}; do
    tag=$(echo "$cfg" | sed 's/[,=/]/_/g')
    envs=$( [ "$cfg" = "-" ] || echo "$cfg" | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py --steps ${STEPS_N:-3} --warmup 1 --no-cpu-baseline \
      --no-gate-sample ${BENCH_ARGS} > "$OUT/b_${tag}_$r.log" 2>&1 || { tail -5 "$OUT/b_${tag}_$r.log"; exit 1; }
    python3 - "$OUT/b_${tag}_$r.log" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], d["value"], "gates/s", {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01})
PY
  done
done
