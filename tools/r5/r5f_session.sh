#!/bin/bash
# Round 5f: the full default bench line (C2 n = 28: GPU step, single-gate sweep, dense gates,
# C3, ABI path, CPU baseline = the whole 20-layer step), then the streaming probe (in place
# vs out of place).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5f
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
tail -c 800 "$OUT/bench.json"; echo
timeout -k 10 120 tools/bin/stream_probe > "$OUT/stream_probe.txt" 2>&1 || exit $?
cat "$OUT/stream_probe.txt"
