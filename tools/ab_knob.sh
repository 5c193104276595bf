#!/bin/bash
# Same-box interleaved A/B of a runtime knob on the bench workload:
#   KNOB=QDC_RQ_PERM_LOW VALS="4 6 8" bash tools/ab_knob.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_${KNOB}; mkdir -p $O
for r in 1 2; do
  for v in $VALS; do
    env $KNOB=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gate-sample > $O/${v}_$r.log 2>&1 || exit $?
    echo "$KNOB=$v run $r: $(grep -o '"value": [0-9.]*' $O/${v}_$r.log | head -1) rev $(grep -o '"avg_launch_ms": [0-9.]*' $O/${v}_$r.log | head -1)"
  done
done
