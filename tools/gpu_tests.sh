#!/bin/bash
# GPU parity tests with their printed measurements (floors, drift), the n = 33 full-size C5 test
# last and on its own time limit.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-tests}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_FULL" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_drift.py::test_c5_full_size_10k_gates -x -v -s \
    --timeout 800 --timeout-method thread > "$OUT/c5_full.log" 2>&1
  rc=$?; grep -E "drift|\[fd\]|passed|failed" "$OUT/c5_full.log" | tail -5; exit $rc
fi
