#!/bin/bash
# Mirrored sweeps on by default: the GPU suite, the C2 A/B against QDC_MIRROR=0, then builds
# with plain (not nontemporal) loads / stores: the single-gate weak cells and the C2 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -2; [ $rc -eq 0 ] || exit $rc
grep -c "passes-by ATOL" "$OUT/tests.log"
TAG=${TAG:-r4j}/ab REPS=2 STEPS_N=5 CFGS="- QDC_MIRROR=0 QDC_DEFER_Q1=0" bash tools/ab_env.sh || exit $?
for v in lib exp/ntld0 exp/ntst0 exp/nt00; do
  if [ $v = lib ]; then d=""; else d="$PWD/$v"; fi
  tag=$(echo $v | tr '/' '_')
  QDC_LIB_DIR=$d QDC_SRC_DIR=$PWD/differentiable-quantum-circuit-cuda_amd/csrc timeout -k 10 300 \
    python3 -u tools/micro_tune.py --reps 1 --q1 1,20,24 --q2 5:20,26:27 --cfgs "-" --out "$OUT/micro_$tag.json" \
    > "$OUT/micro_$tag.log" 2>&1 || exit $?
  grep -E "apply|reverse" "$OUT/micro_$tag.log" | sed "s|^|$v |"
  QDC_LIB_DIR=$d QDC_SRC_DIR=$PWD/differentiable-quantum-circuit-cuda_amd/csrc timeout -k 10 300 \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/bench_$tag.log" 2>&1 || exit $?
  python3 -c "
import json,sys
d=json.loads([l for l in open('$OUT/bench_$tag.log') if l.startswith('{')][-1])
print('$v', d['value'], {k:(v['launches'],v['avg_ms']) for k,v in d['kernels'].items() if v['share']>0.01})"
done
