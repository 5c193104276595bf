#!/bin/bash
# Round 5a: mirrored reverse sweeps on sharded circuits (unremap) — the mirror / sharded /
# configs GPU suites, then one bench line of the library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5a
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_sharded.py tests/test_gpu_configs.py \
  -x -v -s --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -c 600 "$OUT/bench.json"; exit $rc
