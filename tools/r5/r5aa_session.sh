#!/bin/bash
# Round 5aa: the Gamma reduce-scatter's share of fused_reverse (timing-only ablation bit 8:
# Gamma accumulated but not reduced across the wave), same box as the production library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5aa
mkdir -p "$OUT"
export TMPDIR=/tmp
PKG=differentiable-quantum-circuit-cuda_amd
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], d["value"], "gates/s", {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01})
PY
}
for v in base 8 base 8; do
  if [ $v = base ]; then
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $?
  else
    QDC_BENCH_ABLATION=1 QDC_LIB_DIR=$PWD/$PKG/lib-abl$v timeout -k 10 400 python bench.py --steps 3 --warmup 1 \
      --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $?
  fi
  summ "$OUT/b_$v.log" "abl$v"
done
