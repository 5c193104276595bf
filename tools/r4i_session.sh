#!/bin/bash
# Stage algebra split (wide type for the applied products only): GPU parity of the circuits in
# both precisions and both sweep modes, the pass structure of C2 per mode (QDC_RQ_STATS: stages
# and ops per register-resident pass), C3 host times; then the dense-gate / single-gate session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_drift.py tests/test_gpu_circuit.py tests/test_gpu_fusion.py \
  -x -v -s --timeout 300 --timeout-method thread -k "not ablation" \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; grep -E "uncomputed|passed|failed" "$OUT/tests.log" | tail -24; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  QDC_MIRROR=$m QDC_RQ_STATS=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gate-sample \
    > "$OUT/stats_m$m.log" 2> "$OUT/stats_m$m.err" || exit $?
done
grep -c "rq pass" "$OUT"/stats_m*.err
timeout -k 10 300 python3 tools/vqse_once.py > "$OUT/c3.log" 2>&1; tail -c 500 "$OUT/c3.log"; echo
TAG=${TAG:-r4i}/h bash tools/r4h_session.sh
