#!/bin/bash
# VALU instruction mix of the fused kernels on the C2 bench (20 layers, 1 step): one rocprofv3
# --pmc pass per counter set (at most 8 SQ counters each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-mix}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"
P2="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU"
P3="SQ_INSTS_VALU_FLOPS_FP32 SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/rq1_p$i" -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-gate-sample ${BENCH_ARGS} \
    > "$OUT/rq1_p$i.log" 2>&1 || exit $?
done
python3 tools/sq_summary.py "$OUT"
