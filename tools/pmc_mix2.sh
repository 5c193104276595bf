#!/bin/bash
# Instruction mix of the fused kernels (two SQ counter passes, kernel trace only) per variant.
# VARIANTS: "name:libdir" (libdir "-" = the product library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-mix2}
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES"
for v in ${VARIANTS:-prod:-}; do
  name=${v%%:*}; lib=${v#*:}
  if [ "$lib" = "-" ]; then envs=""; else envs="QDC_LIB_DIR=$lib QDC_BENCH_ABLATION=1"; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    env $envs timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/${name}_p$i" -o run \
      -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/${name}_p$i.log" 2>&1 || exit 1
  done
done
echo done
