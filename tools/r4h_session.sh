#!/bin/bash
# Dense k-qubit kernels (tools/r4_qk.sh: pipelining A/B, parity, kernel trace, PMC) and the
# single-gate knob sweep at the sweep's weak cells (tools/micro_tune.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4h}
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${TAG:-r4h}/qk bash tools/r4_qk.sh || exit $?
timeout -k 10 900 python3 -u tools/micro_tune.py --reps 2 --out "$OUT/micro_tune.json" \
  --cfgs "- QDC_XCD_MAP=0 QDC_DIRECT_IT=2 QDC_DIRECT_IT=4 QDC_TILE_FAR=3 QDC_TILE_FAR=7 QDC_TILE1_WIDE=1,QDC_TILE_FAR=3 QDC_GRID_CAP=65536" \
  > "$OUT/micro_tune.log" 2>&1 || exit $?
tail -80 "$OUT/micro_tune.log"
