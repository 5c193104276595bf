#!/bin/bash
# Round 5o: relayout LDS swizzle searched over the C2 relayouts (rq_swz): parity, same-box C2
# A/B against the k_fused swizzle (QDC_RQ_SWZ=0), LDS bank-conflict counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5o
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_mirror.py -x -q --timeout 300 --timeout-method thread \
  > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], d["value"], "gates/s", d["ms_per_step"], "ms/step", {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01}, "compiled", d["ranks"][0].get("kernels_compiled"))
PY
}
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample"
i=0
for v in new old new old; do
  i=$((i+1))
  if [ $v = old ]; then E="QDC_RQ_SWZ=0"; else E="QDC_RQ_SWZ=1"; fi
  env $E timeout -k 10 400 $B > "$OUT/b_${v}_$i.log" 2>&1 || { tail -5 "$OUT/b_${v}_$i.log"; exit 1; }
  summ "$OUT/b_${v}_$i.log" $v
done
P2="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
for v in new old; do
  if [ $v = old ]; then export QDC_RQ_SWZ=0; else export QDC_RQ_SWZ=1; fi
  timeout -s KILL 150 rocprofv3 --pmc $P2 --output-format csv -d "$OUT/sq_$v" -o pmc \
    -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gate-sample \
    > "$OUT/sq_$v.log" 2>&1 || exit $?
done
unset QDC_RQ_SWZ
python3 tools/sq_summary.py "$OUT/sq_new" > "$OUT/sq_new.txt" 2>&1; python3 tools/sq_summary.py "$OUT/sq_old" > "$OUT/sq_old.txt" 2>&1
grep -h "fused_reverse\|fused_apply" "$OUT/sq_new.txt" "$OUT/sq_old.txt" | cut -c1-400
