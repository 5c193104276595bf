#!/bin/bash
# Pass structure and SQ / clock counters of the committed library's fused kernels at C2 n = 28:
# the register-resident pass programs (QDC_RQ_STATS=2: stages, ops and stage lists per pass),
# two SQ counter passes and one clock pass (one rocprofv3 run each).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
QDC_RQ_STATS=2 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-gate-sample \
  > "$OUT/stats.log" 2> "$OUT/stats.err" || exit $?
RQS=1 TAG=${TAG:-prof}/sq bash tools/pmc_sq.sh > "$OUT/sq.txt" 2>&1 || exit $?
TAG=${TAG:-prof}/clock bash tools/pmc_clock.sh > "$OUT/clock.txt" 2>&1 || exit $?
echo done
