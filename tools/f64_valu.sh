#!/bin/bash
# f64 path (config C3, VQSE n = 26): dynamic instruction counts of the fused kernels (one
# rocprofv3 --pmc pass per counter set over tools/vqse_once.py), summary per kernel
# (tools/sq_summary.py).  QDC_LIB_DIR passes through (A/B builds).  Time-boxed steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-f64valu}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/rq1_p$i" -o pmc \
    -- python3 tools/vqse_once.py > "$OUT/rq1_p$i.log" 2>&1 || exit $?
done
python3 tools/sq_summary.py "$OUT"
