#!/bin/bash
# Same-box A/B of runtime knobs on config C3 (VQSE n = 26 f64, tools/vqse_once.py: seconds per
# loss-and-gradient call): CFGS as tools/ab_env.sh (comma separated VAR=VALUE, "-" defaults),
# interleaved REPS times.  Time-boxed steps; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-c3_env_ab}
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-2}); do
  for cfg in ${CFGS:--}; do
    tag=$(echo "$cfg" | sed 's/[,=/]/_/g')
    envs=$( [ "$cfg" = "-" ] || echo "$cfg" | tr ',' ' ')
    env $envs timeout -k 10 300 python3 tools/vqse_once.py > "$OUT/c3_${tag}_$r.log" 2>&1 || { tail -5 "$OUT/c3_${tag}_$r.log"; exit 1; }
    echo "$cfg run $r: $(head -c 160 "$OUT/c3_${tag}_$r.log")"
  done
done
