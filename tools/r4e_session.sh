#!/bin/bash
# Round-4 GPU session: the GPU parity suite (default configuration), the fused tests with
# one-wave 2^11 forward tiles, the mirrored-sweep tests (a numerical failure there does not stop
# the session; a crash does), then an interleaved C2 A/B of the round's runtime options.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates --ignore tests/test_gpu_mirror.py \
  > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -2; [ $rc -eq 0 ] || exit $rc
QDC_TILE1_CHUNKS=1024 QDC_RW=11 timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_circuit.py \
  -k "not ablation" -x -q --timeout 300 --timeout-method thread > "$OUT/tests_t1k.log" 2>&1
rc=$?; tail -1 "$OUT/tests_t1k.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_mirror.py -v -s --timeout 300 --timeout-method thread \
  > "$OUT/tests_mirror.log" 2>&1
rc=$?; grep -E "passes-by|passed|failed" "$OUT/tests_mirror.log" | tail -40; [ $rc -le 1 ] || exit $rc
TAG=${TAG:-r4e}/ab REPS=2 STEPS_N=5 CFGS="- QDC_TILE1_CHUNKS=1024,QDC_RW=3 QDC_TILE1_CHUNKS=1024,QDC_RW=11 QDC_DIAG_INJECT=0 QDC_SCHED_CACHE=0 QDC_MIRROR=1" bash tools/ab_env.sh
