#!/bin/bash
# Round 5q: register-resident tile order (QDC_RQ_ORDER: 0 block-contiguous, 1 grid-strided so
# concurrently running tiles are neighbours in memory, 2 block-contiguous in XCD-aware order)
# on the C2 step, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5q
mkdir -p "$OUT"
export TMPDIR=/tmp
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], d["value"], "gates/s", d["ms_per_step"], "ms/step", {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01})
PY
}
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample"
i=0
for v in 0 1 2 0 1 2; do
  i=$((i+1))
  QDC_RQ_ORDER=$v timeout -k 10 300 $B > "$OUT/b_o${v}_$i.log" 2>&1 || { tail -5 "$OUT/b_o${v}_$i.log"; exit 1; }
  summ "$OUT/b_o${v}_$i.log" "order$v"
done
