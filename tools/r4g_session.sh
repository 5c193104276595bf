#!/bin/bash
# Mirrored sweeps with densities after the gates of a pass: GPU parity (mirror tests, fusion),
# then an interleaved C2 A/B default vs QDC_MIRROR=1 and the C3 (f64) call with host times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4g}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mirror.py -v -s --timeout 300 --timeout-method thread \
  > "$OUT/tests_mirror.log" 2>&1
rc=$?; grep -E "uncomputed|passed|failed" "$OUT/tests_mirror.log" | tail -12; [ $rc -le 1 ] || exit $rc
QDC_MIRROR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_circuit.py tests/test_gpu_drift.py -x -q --timeout 300 --timeout-method thread \
  -k "not ablation" --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests_m1.log" 2>&1
rc=$?; tail -2 "$OUT/tests_m1.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 tools/vqse_once.py > "$OUT/c3.log" 2>&1; tail -c 600 "$OUT/c3.log"; echo
QDC_MIRROR=1 timeout -k 10 300 python3 tools/vqse_once.py > "$OUT/c3_m1.log" 2>&1; tail -c 600 "$OUT/c3_m1.log"; echo
TAG=${TAG:-r4g}/ab REPS=2 STEPS_N=5 CFGS="- QDC_MIRROR=1" bash tools/ab_env.sh
