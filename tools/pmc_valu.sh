#!/bin/bash
# Dynamic instruction mix of the fused kernels at the bench's own configuration (C2, n = 28,
# 20 layers): one rocprofv3 --pmc pass per counter set (SQ <= 8, GRBM <= 2), each time-boxed.
# Summary per kernel: tools/sq_summary.py.  QDC_LIB_DIR / extra env pass through (A/B builds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-valu}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
P2="SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P3="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d "$OUT/rq1_p$i" -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 ${BENCH_ARGS} --no-cpu-baseline --no-gate-sample \
    > "$OUT/rq1_p$i.log" 2>&1 || exit $?
done
python3 tools/sq_summary.py "$OUT"
