#!/bin/bash
# Round 6x (final library: single-gate reverse kernels, address-map exceptions, early injections): smoke(), the whole GPU suite, C5 at n = 33.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6x
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -3 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_drift.py::test_c5_full_size_10k_gates -x -v -s \
  --timeout 480 --timeout-method thread > "$OUT/c5_full.log" 2>&1
rc=$?; grep -E "drift|\[fd\]|passed|failed" "$OUT/c5_full.log" | tail -5; exit $rc
