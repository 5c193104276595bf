#!/bin/bash
# Round 6e: the dynamic tail's granule (QDC_DYN_GRAN: fewer granule partials for k_dsum to
# pre-sum) — same-box A/B of the bench step, and the dynamic-tail determinism test at the
# candidate granule; then the GPU suite on this library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6e
mkdir -p "$OUT"
export TMPDIR=/tmp
QDC_DYN_GRAN=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py -k "dynamic_tail or specialized_passes_equal" \
  -x -v --timeout 240 --timeout-method thread > "$OUT/tests_gran8.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests_gran8.log" | tail -2; [ $rc -eq 0 ] || exit $rc
for g in 1 4 8 16 1 4 8 16; do
  QDC_DYN_GRAN=$g timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 \
    --no-cpu-baseline --no-gate-sample > "$OUT/bench_gran$g.json" 2> "$OUT/bench_gran$g.err" || exit $?
  python3 -c "
import json; s=open('$OUT/bench_gran$g.json').read(); L=json.loads(s[s.index('{\"metric\"'):].splitlines()[0])
k=L['kernels']; print('gran $g', L['value'], L['ms_per_step'], 'rev', k['fused_reverse']['avg_ms'], 'apply', k['fused_apply']['avg_ms'], 'copy', k.get('copy',{}).get('avg_ms'), 'set_standard', k.get('set_standard',{}).get('avg_ms'))" | tee -a "$OUT/gran_ab.txt"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3; exit $rc
