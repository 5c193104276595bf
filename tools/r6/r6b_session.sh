#!/bin/bash
# Round 6b: density-only passes on k_dens1 + forward passes split into gates / densities
# (QDC_DENS1, QDC_DENS_SPLIT).  The whole GPU suite (fusion tests first), C5 at n = 33, the
# bench line, then the rocprofv3 kernel trace + stats and the PMC traffic passes of the same
# library (the JIT fingerprint no longer changes under the profiler).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6b
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fusion.py tests -m gpu -x -v --timeout 400 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -c 400 "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/trace.log" 2>&1
rc=$?; tail -c 300 "$OUT/trace.log"; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_agg.py "$OUT/trace/trace_kernel_stats.csv" > "$OUT/kernel_stats_by_bench_name.csv" || exit $?
head -8 "$OUT/kernel_stats_by_bench_name.csv"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-gate-sample > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT" "$OUT/summary" > "$OUT/pmc_summary.log" 2>&1 || exit $?
tail -5 "$OUT/pmc_summary.log"
timeout -k 10 500 python -u -m pytest tests/test_gpu_drift.py::test_c5_full_size_10k_gates -x -v -s \
  --timeout 480 --timeout-method thread > "$OUT/c5_full.log" 2>&1
rc=$?; grep -E "drift|\[fd\]|passed|failed" "$OUT/c5_full.log" | tail -5; exit $rc
