#!/bin/bash
# Counter passes (one rocprofv3 --pmc run per set, short C2 bench) for the fused kernels; the
# sets are given one per argument.  Summaries per kernel: tools/sq_summary.py gpurun_out/$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/rq1_p$i" -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --layers 4 --no-cpu-baseline --no-gate-sample \
    > "$OUT/rq1_p$i.log" 2>&1 || exit $?
done
python3 tools/sq_summary.py "$OUT"
