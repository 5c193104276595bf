#!/bin/bash
# Round 5w: the fused passes' tile pattern by row length and waves per SIMD (stream_probe3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r5w
timeout -k 10 200 tools/bin/stream_probe3 > gpurun_out/r5w/stream_probe3.txt 2>&1; rc=$?
cat gpurun_out/r5w/stream_probe3.txt; exit $rc
