#!/bin/bash
# Round 6a: the new and changed GPU suites (C5 at n = 26 on 8 shards / 2 streams, C3 in both
# precisions with floors, the mirror suite's 2-norm lines), then the bench line (C2 headline with
# the vqse_c3_f32 block) and the 8-local-shard rehearsal line (exchange block).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6a
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_c5_shards.py tests/test_gpu_vqse.py tests/test_gpu_mirror.py \
  -x -v -s --timeout 600 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -c 300 "$OUT/bench.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --local-shards 8 > "$OUT/bench_shards8.json" 2> "$OUT/bench_shards8.err"
rc=$?; tail -c 600 "$OUT/bench_shards8.json"; [ $rc -eq 0 ] || exit $rc
# per-dispatch trace of one C2 step (the per-pass time model of fused_reverse: joined by launch
# order with the dry-run census of the same program, tools/r6/pass_model.py)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o trace \
  -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/trace.log" 2>&1
rc=$?; tail -c 300 "$OUT/trace.log"; exit $rc
