#!/bin/bash
# Round 5y: config C4 on one GPU (brickwall, n = 30, 40 layers, f32) as a bench line: the warm-up runs
# the interpreted passes while its ~270 specialized kernels compile in the background; the
# bench waits for them (progress on stderr), then times one step on the specialized passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5y
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1120 python -u bench.py --workload c4 --steps 1 --warmup 1 --no-gate-sample \
  > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || { tail -20 "$OUT/bench_c4.err"; exit 1; }
tail -c 1500 "$OUT/bench_c4.json"; echo
