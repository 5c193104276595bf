#!/bin/bash
# f64 path (config C3, VQSE n = 26): rocprofv3 kernel trace + stats, and FETCH_SIZE /
# WRITE_SIZE passes (separate runs) of one tools/vqse_once.py invocation; summary by
# tools/pmc_summary.py --detail-only.  Every GPU step time-boxed; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-f64}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/f64_trace" -o trace \
  -- python3 tools/vqse_once.py > "$OUT/f64_trace.log" 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/f64_pmc_$c" -o pmc \
    -- python3 tools/vqse_once.py > "$OUT/f64_pmc_$c.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT" "$OUT/f64" --prefix f64_ --detail-only > "$OUT/f64_pmc_summary.log" 2>&1
