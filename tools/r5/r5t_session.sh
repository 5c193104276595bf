#!/bin/bash
# Round 5t: the full default bench line with the final library (C2 n = 28: GPU step, single-gate
# sweep, dense gates, C3, ABI path, CPU baseline = the whole 20-layer step), then the shard
# rehearsal (local shards / shard streams on one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5t
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
tail -c 600 "$OUT/bench.json"; echo
TAG=r5t/shard bash tools/shard_rehearsal.sh
