#!/bin/bash
# Same-box A/B of f64 builds on config C3 (VQSE n = 26, tools/vqse_once.py: seconds per
# loss-and-gradient call): LIBS ("lib" = in-tree, else a build directory holding
# libqdc_f64.so), interleaved REPS times.  Time-boxed steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-c3_ab}
mkdir -p "$OUT"
for r in $(seq 1 ${REPS:-2}); do
  for l in $LIBS; do
    tag=$(echo $l | tr '/' '_')
    if [ "$l" = lib ]; then d=""; else d="$PWD/$l"; fi
    QDC_LIB_DIR=$d timeout -k 10 300 python3 tools/vqse_once.py > "$OUT/${tag}_$r.log" 2>&1 || exit $?
    echo "$l run $r: $(head -c 160 "$OUT/${tag}_$r.log")"
  done
done
