#!/bin/bash
# Round 5z: the final bench line and the rocprofv3 kernel trace of the same workload on the same
# box (the line's live per-kernel HIP-event times and rocprofv3's must agree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5z
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
tail -c 400 "$OUT/bench.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/trace.log" 2>&1 || exit $?
tail -1 "$OUT/trace.log" | tail -c 300
