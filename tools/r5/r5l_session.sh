#!/bin/bash
# Round 5l: LANE family with units in flight (U) and the diagonal reverse with 8 chunks in
# flight: parity (default knobs and U=1,4,8 / diag 2), then single-gate sweeps by knob set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5l
mkdir -p "$OUT"
export TMPDIR=/tmp
T="tests/test_gpu_lane.py tests/test_gpu_primitives.py tests/test_gpu_golden.py tests/test_gpu_abi_replay.py tests/test_gpu_fusion.py::test_fused_equals_unfused_and_oracle"
timeout -k 10 300 python -u -m pytest $T -q --timeout 240 --timeout-method thread \
  > "$OUT/tests_default.log" 2>&1 || { grep -E "failing cells|passed|failed|Error" "$OUT/tests_default.log" | cut -c1-3000; exit 1; }
tail -1 "$OUT/tests_default.log"
QDC_LANE_U=1,4,8 QDC_DIAG_RU=2 timeout -k 10 300 python -u -m pytest $T -q --timeout 240 --timeout-method thread \
  > "$OUT/tests_u148.log" 2>&1 || { grep -E "failing cells|passed|failed|Error" "$OUT/tests_u148.log" | cut -c1-3000; exit 1; }
tail -1 "$OUT/tests_u148.log"
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --micro > "$OUT/micro_$tag.log" 2>&1 || { tail -20 "$OUT/micro_$tag.log"; exit 1; }
}
run l7_841 QDC_LANE=7
run l2_d2 QDC_LANE=2 QDC_DIAG_RU=2
run l7_414 QDC_LANE=7 QDC_LANE_U=4,4,4
run l7_888 QDC_LANE=7 QDC_LANE_U=8,8,8
run l7_841b QDC_LANE=7
