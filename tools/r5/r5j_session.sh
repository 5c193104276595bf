#!/bin/bash
# Round 5j: the GPU suite with the LANE family on (k_lane: single-gate ops with one chunk per
# lane), then the single-gate sweep (fusion off, n = 28 f32) with QDC_LANE=7 / 0 / 7 on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5j
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
for v in 7 0 7; do
  QDC_LANE=$v timeout -k 10 300 python -u bench.py --micro > "$OUT/micro_lane$v.log" 2>&1 || { tail -20 "$OUT/micro_lane$v.log"; exit 1; }
  cp "$OUT/micro_lane$v.log" "$OUT/micro_lane${v}_$(date +%s).log"
done
