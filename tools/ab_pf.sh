#!/bin/bash
# GPU session: parity tests, then A/B of the register-prefetch variants of k_rq on the C2 bench
# (QDC_RQ_PF one-state, QDC_RQ_PF2 two-state).  Every GPU step is time-boxed; the chain stops at
# the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_pf}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for cfg in "1 1" "0 0" "1 0" "1 1"; do
  set -- $cfg
  echo "== PF=$1 PF2=$2"
  QDC_RQ_PF=$1 QDC_RQ_PF2=$2 timeout -k 10 300 python bench.py --steps 5 --warmup 2 \
    --no-cpu-baseline --no-gate-sample > "$OUT/bench_$1$2.log" 2>&1 || exit $?
  python3 - "$OUT/bench_$1$2.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(d["value"], "gates/s", d["ms_per_step"], "ms/step",
      {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01})
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/trace.log" 2>&1 || exit $?
echo done
