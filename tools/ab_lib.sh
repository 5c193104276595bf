#!/bin/bash
# Same-box interleaved A/B of two builds of the library on the bench workload:
#   LIBS="build/base lib" bash tools/ab_lib.sh   ("lib" = the in-tree build)
# Each run prints gates/s and the per-launch ms of the fused kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_lib; mkdir -p $O
ARGS=${ARGS:-"--steps 8 --warmup 2 --no-cpu-baseline --no-gate-sample"}
for r in 1 2; do
  for l in $LIBS; do
    tag=$(echo $l | tr '/' '_')
    if [ "$l" = lib ]; then d=""; else d="$PWD/$l"; fi
    QDC_LIB_DIR=$d timeout -k 10 300 python bench.py $ARGS > $O/${tag}_$r.log 2>&1 || exit $?
    python3 - $O/${tag}_$r.log $l $r <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
k = d["kernels"]
print(f"{sys.argv[2]:>14s} run {sys.argv[3]}: {d['value']:8.1f} gates/s  " +
      "  ".join(f"{n} {k[n]['avg_ms']:.4f}" for n in ("fused_reverse", "fused_apply", "fused_inject") if n in k))
PY
  done
done
