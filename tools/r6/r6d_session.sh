#!/bin/bash
# Round 6d: timing-only profiler events (hipEventDisableSystemFence) — same-box A/B of the bench
# step against default events (QDC_EVENT_FENCE=1) with unprofiled steps beside each; the diagonal
# kernels' XCD block order (QDC_XCD_MAP bit 2) on the single-gate cells; then the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6d
mkdir -p "$OUT"
export TMPDIR=/tmp
for f in 0 1 0 1; do
  QDC_EVENT_FENCE=$f QDC_BENCH_UNPROFILED_STEPS=10 timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 \
    --no-cpu-baseline --no-gate-sample > "$OUT/bench_fence$f.json" 2> "$OUT/bench_fence$f.err" || exit $?
  python3 -c "
import json,sys; s=open('$OUT/bench_fence$f.json').read(); L=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
print('fence $f', L['value'], L['ms_per_step'], 'unprofiled', L['unprofiled_ms_per_step'], 'rev', L['kernels']['fused_reverse']['avg_ms'], 'apply', L['kernels']['fused_apply']['avg_ms'])" | tee -a "$OUT/fence_ab.txt"
done
for x in 1 5 1 5; do
  QDC_XCD_MAP=$x timeout -k 10 300 python -u tools/r5/micro_subset.py --q1 0,20 \
    --q2 0:1,5:20,26:27,14:13 > "$OUT/micro_xcd$x.log" 2>&1 || exit $?
  echo "xcd $x $(grep -E 'reverse_q2_diag|apply_q2_diag' "$OUT/micro_xcd$x.log" | awk '{for(i=1;i<=NF;i++) if($i ~ /%$/) p=$i; print $1$2,$3,p}' | tr '\n' ' ')" | tee -a "$OUT/diag_xcd_ab.txt"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3; exit $rc
