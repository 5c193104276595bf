#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r4f
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_drift.py tests/test_gpu_circuit.py -v -s --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; grep -E "uncomputed|passed|failed" "$OUT/tests.log" | tail -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/vqse_once.py > "$OUT/c3.log" 2>&1; tail -c 400 "$OUT/c3.log"
