#!/bin/bash
# Round 5s (final library): the whole GPU suite (C5 n = 33 on its own time limit), PMC traffic passes and the
# rocprofv3 kernel trace of the bench workload with the library of this commit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_drift.py::test_c5_full_size_10k_gates -x -v -s \
  --timeout 380 --timeout-method thread > "$OUT/c5_full.log" 2>&1
rc=$?; grep -E "drift|\[fd\]|passed|failed" "$OUT/c5_full.log" | tail -5; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-gate-sample > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT" "$OUT/summary" > "$OUT/pmc_summary.log" 2>&1 || exit $?
tail -5 "$OUT/pmc_summary.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/trace.log" 2>&1 || exit $?
tail -c 400 "$OUT/trace.log"
