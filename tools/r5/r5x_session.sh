#!/bin/bash
# Round 5x: dynamic-tail static share down to 0 (all tiles from the per-XCD counters), same box: dynamic
# tail static share (QDC_DYN), permuting passes' low positions (QDC_RQ_PERM_LOW), same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5x
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
for v in "QDC_DYN=35" "QDC_DYN=0" "QDC_DYN=10" "QDC_DYN=35" "QDC_DYN=0" "QDC_DYN=10"; do
  i=$((i+1))
  env $v timeout -k 10 300 $B > "$OUT/b_$i.log" 2>&1 || { tail -5 "$OUT/b_$i.log"; exit 1; }
  summ "$OUT/b_$i.log" "$v"
done
