#!/bin/bash
# Round 6k: diagonal reverse with k fixed per thread (k_diag_q, QDC_DIAG_Q=1) against k_diag
# (QDC_DIAG_Q=0) on the single-gate cells, interleaved; then the diagonal reverse parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6k
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py -x -v --timeout 200 --timeout-method thread \
  -k "diag_reverse or every_op_class" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
for x in 0 1 0 1; do
  QDC_DIAG_Q=$x timeout -k 10 300 python -u tools/r5/micro_subset.py --q1 0 \
    --q2 0:1,5:20,26:27,14:13,3:9 > "$OUT/micro_q$x.log" 2>&1 || exit $?
  echo "diag_q $x $(grep -E 'reverse_q2_diag' "$OUT/micro_q$x.log" | awk '{for(i=1;i<=NF;i++) if($i ~ /%$/) p=$i; print $3,p}' | tr '\n' ' ')" | tee -a "$OUT/diag_q_ab.txt"
done
grep -E "passed|failed" "$OUT/tests.log" | tail -2
