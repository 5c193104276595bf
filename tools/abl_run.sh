#!/bin/bash
# GPU: bench the ablation builds (tools/ablate.sh) against the product build, then SQ counter
# passes on the product build.  Time-boxed steps, stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abl}
mkdir -p "$OUT"
export TMPDIR=/tmp
summ() {
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(d["value"], "gates/s", d["ms_per_step"], "ms/step",
      {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01})
PY
}
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
for v in base ${ABLS:-1 2 4 8 16 3}; do
  echo "== $v"
  if [ $v = base ]; then
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $?
  else
    QDC_BENCH_ABLATION=1 QDC_LIB_DIR=build/abl$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
      --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $?
  fi
  summ "$OUT/b_$v.log"
done
RQS=1 TAG=${TAG:-abl}/sq bash tools/pmc_sq.sh > "$OUT/sq.log" 2>&1 || exit $?
cat "$OUT/sq.log"
