#!/bin/bash
# Round 5k: LANE-family parity at every placement, then the single-gate sweep (fusion off,
# n = 28 f32) with QDC_LANE=7 / 0 / 7 on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5k
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_primitives.py tests/test_gpu_golden.py tests/test_gpu_abi_replay.py -q --timeout 240 --timeout-method thread \
  > "$OUT/lane.log" 2>&1 || { grep -E "failing cells|passed|failed|Error" "$OUT/lane.log" | cut -c1-3000; exit 1; }
tail -2 "$OUT/lane.log"
for v in 7 0 7; do
  QDC_LANE=$v timeout -k 10 300 python -u bench.py --micro > "$OUT/micro_lane$v.log" 2>&1 || { tail -20 "$OUT/micro_lane$v.log"; exit 1; }
  cp "$OUT/micro_lane$v.log" "$OUT/micro_lane${v}_$(date +%s).log"
done
