#!/bin/bash
# Round 5b: re-attribution of the fused passes on the kernels that actually run (specialized).
#  1. the ablation triple and single-term ablations: bench (C2 n=28, 3 steps) with the
#     production library and each lib-abl<bits> build (QDC_RQ_ABL: 3 skeleton = no stage math
#     and no relayouts, 32 compute only = no HBM traffic, 2 no relayouts, 4 no Gamma, 1 no
#     stage math) — every one running specialized passes (ranks[0].kernels_compiled > 0);
#  2. the MFMA / VALU co-issue probe, plain and under SQ_VALU_MFMA_COEXEC_CYCLES;
#  3. SQ counters per fused kernel of the production library (LDS bank conflicts, waits).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5b
mkdir -p "$OUT"
export TMPDIR=/tmp
PKG=differentiable-quantum-circuit-cuda_amd
summ() {
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(d["value"], "gates/s", d["ms_per_step"], "ms/step", "compiled", d["ranks"][0]["kernels_compiled"],
      {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01})
PY
}
for v in base 3 32 2 4 1 base; do
  echo "== $v"
  if [ $v = base ]; then
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $?
  else
    QDC_BENCH_ABLATION=1 QDC_LIB_DIR=$PWD/$PKG/lib-abl$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
      --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $?
  fi
  summ "$OUT/b_$v.log"
done
echo "== coissue probe"
timeout -k 10 60 tools/bin/coissue_probe > "$OUT/coissue.txt" 2>&1 || exit $?
cat "$OUT/coissue.txt"
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
  --output-format csv -d "$OUT/coissue_pmc" -o pmc -- tools/bin/coissue_probe > "$OUT/coissue_pmc.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA \
  --output-format csv -d "$OUT/coissue_pmc2" -o pmc -- tools/bin/coissue_probe > "$OUT/coissue_pmc2.log" 2>&1 || exit $?
echo "== membw (in-place streaming vs copy)"
timeout -k 10 120 tools/bin/membw > "$OUT/membw.txt" 2>&1 || exit $?
head -8 "$OUT/membw.txt"
echo "== SQ passes"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/sq/rq1_p$i" -o pmc \
    -- python3 bench.py --steps 1 --warmup 1 --layers 4 --no-cpu-baseline --no-gate-sample \
    > "$OUT/sq_p$i.log" 2>&1 || exit $?
done
python3 tools/sq_summary.py "$OUT/sq" | tee "$OUT/sq_summary.txt"
