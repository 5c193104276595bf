#!/bin/bash
# A GPU session of selected steps (STEPS, space separated; default all): c5full, bench, micro,
# pmc, trace.  Every GPU step is time-boxed; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-session}
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in ${STEPS:-c5full bench micro}; do
  echo "== $s $(date +%T)"
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread \
        --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1 || { tail -20 "$OUT/tests.log"; exit 1; }
      grep -E "passed|failed" "$OUT/tests.log" | tail -1 ;;
    c5full)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_drift.py::test_c5_full_size_10k_gates -x -v -s \
        --timeout 500 --timeout-method thread > "$OUT/c5_full.log" 2>&1 || { tail -20 "$OUT/c5_full.log"; exit 1; }
      grep -E "drift|\[fd\]|passed" "$OUT/c5_full.log" ;;
    bench)
      timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
      tail -c 1500 "$OUT/bench.log"; echo ;;
    micro)
      timeout -k 10 900 python -u bench.py --micro > "$OUT/micro.log" 2>&1 || { tail -20 "$OUT/micro.log"; exit 1; }
      python3 tools/micro_table.py "$OUT/micro.log" | tee "$OUT/micro_table.txt" ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc \
          -- python3 bench.py --steps 1 --warmup 0 --layers 2 --no-cpu-baseline --no-gate-sample > "$OUT/pmc_$c.log" 2>&1 || exit 1
      done
      python3 tools/pmc_summary.py "$OUT" "$OUT/summary" ;;
    trace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
        -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/trace.log" 2>&1 || exit 1
      head -6 "$OUT/trace/trace_kernel_stats.csv" | cut -c1-160 ;;
  esac
done
echo "== done $(date +%T)"
