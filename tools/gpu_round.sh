#!/bin/bash
# One GPU session: parity tests, PMC passes (one counter set per pass, short run) and their
# summary, the full bench (with CPU baseline; it reads this round's PMC traffic), then a
# rocprofv3 kernel trace of the bench workload.  Every GPU step is time-boxed and the chain
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-round}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1"; }
step tests
timeout -k 10 900 python -m pytest tests -m gpu -q > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  step "pmc $c"
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --layers 2 --no-cpu-baseline --no-gate-sample > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
step pmc-summary
python3 tools/pmc_summary.py "$OUT" "$OUT/summary" > "$OUT/pmc_summary.log" 2>&1 || exit $?
step bench
timeout -k 10 900 python bench.py --pmc "$OUT/pmc_traffic.json" > "$OUT/bench.log" 2>&1 || exit $?
tail -c 600 "$OUT/bench.log"; echo
step rocprof-kernel-trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/trace.log" 2>&1 || exit $?
step done
