#!/bin/bash
# Round 5i: gate-shaped streaming patterns by row bit, LDS-exchanged rows and two-state
# reduction grids (stream_probe2), then config C5 on one GPU as a bench line (r5g's command:
# n = 33, 10 000 gates, f32; the specialized kernels compile in the background during warm-up).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5i
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 150 tools/bin/stream_probe2 > "$OUT/stream_probe2.txt" 2>&1 || { cat "$OUT/stream_probe2.txt"; exit 1; }
cat "$OUT/stream_probe2.txt"
timeout -k 10 1000 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-gate-sample \
  > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { tail -20 "$OUT/bench_c5.err"; exit 1; }
tail -c 1500 "$OUT/bench_c5.json"; echo
