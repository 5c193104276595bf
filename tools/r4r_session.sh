#!/bin/bash
# Half-buffer relayouts (one-wave five-slot passes: two rounds through half the LDS buffer,
# plans that keep a register slot): the GPU suite, then the C2 A/B against QDC_SPEC_HALF=0 and
# the C3 call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4r}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" "$OUT/tests.log" | head -20; exit $rc; }
grep -c "passes-by ATOL" "$OUT/tests.log"
TAG=${TAG:-r4r}/ab REPS=2 STEPS_N=5 CFGS="- QDC_SPEC_HALF=0" bash tools/ab_env.sh || exit $?
timeout -k 10 300 python3 tools/vqse_once.py > "$OUT/c3.log" 2>&1; tail -c 300 "$OUT/c3.log"; echo
