#!/bin/bash
# Dense k-qubit kernel variants (pipelined with doubled batches, paired groups at k = 4, grid
# caps) and the C2 step with the Python wrapper's one-pass marshalling.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -m pytest tests/test_gpu_dense.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -5 "$OUT/tests.log"; exit 1; }
QDC_QK_PF=2 QDC_QK_PAIR=2 timeout -k 10 300 python3 -m pytest tests/test_gpu_dense.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests_v.log" 2>&1 || { tail -5 "$OUT/tests_v.log"; exit 1; }
tail -1 "$OUT/tests_v.log"
for rep in 1 2; do
  for cfg in "-" "QDC_QK_PF=2" "QDC_QK_PAIR=2" "QDC_QK_PAIR=2,QDC_QK_PF=1" "QDC_QK_PAIR=2,QDC_QK_PF=2" "QDC_QK_GRID=8192" "QDC_QK_GRID=2048"; do
    envs=$( [ "$cfg" = "-" ] || echo "$cfg" | tr ',' ' ')
    echo "$cfg $(env $envs timeout -k 10 120 python3 tools/qk_once.py 2>&1 | tail -1)"
  done
done > "$OUT/qk_ab.log"; cat "$OUT/qk_ab.log"
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/bench.log" 2>&1 || exit $?
tail -c 1500 "$OUT/bench.log"
