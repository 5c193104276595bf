#!/bin/bash
# Round 6y (final library: single-gate reverse kernels, address-map exceptions, early injections): the bench line as the driver runs it, its rocprofv3 kernel trace +
# stats (by bench name) and PMC traffic passes, the 8-local-shard rehearsal line and a C4 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6y
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -c 300 "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
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
tail -9 "$OUT/pmc_summary.log"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --local-shards 8 > "$OUT/bench_shards8.json" 2> "$OUT/bench_shards8.err"
rc=$?; tail -c 300 "$OUT/bench_shards8.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-gate-sample > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
rc=$?; tail -c 300 "$OUT/bench_c4.json"; exit $rc
