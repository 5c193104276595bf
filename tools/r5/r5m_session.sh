#!/bin/bash
# Round 5m: block-wide LANE variant (k_lane_blk) for far targets: parity, then single-gate
# sweeps with QDC_LANE_BLK=1 / 0 / 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5m
mkdir -p "$OUT"
export TMPDIR=/tmp
T="tests/test_gpu_lane.py tests/test_gpu_primitives.py tests/test_gpu_golden.py tests/test_gpu_abi_replay.py tests/test_gpu_fusion.py::test_fused_equals_unfused_and_oracle"
timeout -k 10 300 python -u -m pytest $T -q --timeout 240 --timeout-method thread \
  > "$OUT/tests_default.log" 2>&1 || { grep -E "failing cells|passed|failed|Error" "$OUT/tests_default.log" | cut -c1-3000; exit 1; }
tail -1 "$OUT/tests_default.log"
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --micro > "$OUT/micro_$tag.log" 2>&1 || { tail -20 "$OUT/micro_$tag.log"; exit 1; }
}
run blk1 QDC_LANE_BLK=1
run blk0 QDC_LANE_BLK=0
run blk1b QDC_LANE_BLK=1
