#!/bin/bash
# Dense k-qubit MFMA kernels at n = 28 f32: the software-pipelining A/B (QDC_QK_PF), the GPU
# parity tests with it on, a rocprofv3 kernel trace + stats of one sample, FETCH_SIZE /
# WRITE_SIZE passes and one SQ pass (separate runs).  Every GPU step time-boxed; stops at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4qk}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/qk_probe.py --pf > "$OUT/qk_pf_ab.log" 2>&1 || exit $?
cat "$OUT/qk_pf_ab.log"
QDC_QK_PF=1 timeout -k 10 300 python3 -m pytest tests/test_gpu_dense.py -x -q --timeout 120 --timeout-method thread \
  > "$OUT/tests_pf.log" 2>&1 || { tail -5 "$OUT/tests_pf.log"; exit 1; }
tail -1 "$OUT/tests_pf.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
  -- python3 tools/qk_once.py > "$OUT/trace.log" 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o pmc \
    -- python3 tools/qk_once.py > "$OUT/pmc_$c.log" 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/sq" -o pmc -- python3 tools/qk_once.py > "$OUT/sq.log" 2>&1 || exit $?
echo done
