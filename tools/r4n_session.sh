#!/bin/bash
# Round-4 profile session of the committed library: GPU suite (without the n = 33 test), HBM
# traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs) and their summary, the full bench
# (reads this build's traffic), and a rocprofv3 kernel trace + stats of the bench workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4n}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c"
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --layers 2 --no-cpu-baseline --no-gate-sample > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT" "$OUT/summary" > "$OUT/pmc_summary.log" 2>&1 || exit $?
echo "== bench"
timeout -k 10 900 python -u bench.py --pmc "$OUT/pmc_traffic.json" > "$OUT/bench.log" 2> "$OUT/bench.err" || exit $?
tail -c 400 "$OUT/bench.log"; echo
echo "== trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/trace.log" 2>&1 || exit $?
echo done
