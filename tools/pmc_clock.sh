#!/bin/bash
# Effective shader clock and VALU activity of the fused kernels per library variant
# (MI355X_MICROARCH.md "DVFS give-back": clock = GRBM_GUI_ACTIVE / 8 / kernel wall time).
# VARIANTS: space separated "name:libdir" (libdir "-" = the product library).  One counter
# pass with kernel trace per variant (no other trace domains), then tools/pmc_clock.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-clock}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in ${VARIANTS:-prod:-}; do
  name=${v%%:*}; lib=${v#*:}
  if [ "$lib" = "-" ]; then envs=""; else envs="QDC_LIB_DIR=$lib QDC_BENCH_ABLATION=1"; fi
  env $envs timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
    --kernel-trace --output-format csv -d "$OUT/$name" -o run \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/$name.log" 2>&1 || exit 1
done
python3 tools/pmc_clock.py "$OUT" ${VARIANTS:-prod:-}
