#!/bin/bash
# SQ counter passes (one counter set per rocprofv3 run) over a short bench of the C2 workload,
# for the register-resident (QDC_RQ=1) and LDS-resident (QDC_RQ=0) fused kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
for rq in ${RQS:-1 0}; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    QDC_RQ=$rq timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/rq${rq}_p$i" -o pmc \
      -- python3 bench.py --steps 1 --warmup 0 --layers 4 --no-cpu-baseline --no-gate-sample \
      > "$OUT/rq${rq}_p$i.log" 2>&1 || exit $?
  done
done
python3 tools/sq_summary.py "$OUT"
