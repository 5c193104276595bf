#!/bin/bash
# Dynamic instruction counts per launch of the fused kernels for several builds of the library
# (LIBS: "lib" = in-tree, else a build directory), one rocprofv3 --pmc pass each (C2 bench step,
# n = 28), then a same-box timing A/B of the same builds (tools/ab_lib.sh).  Time-boxed steps,
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-valu_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
for l in $LIBS; do
  tag=$(echo $l | tr '/' '_')
  if [ "$l" = lib ]; then d=""; else d="$PWD/$l"; fi
  QDC_LIB_DIR=$d timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d "$OUT/$tag" -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-gate-sample > "$OUT/$tag.log" 2>&1 || exit $?
  echo "== $l"
  python3 - "$OUT/$tag" <<'PY'
import csv, sys
from collections import defaultdict
from pathlib import Path
sys.path.insert(0, "tools")
from pmc_summary import bench_name
tot = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(lambda: defaultdict(int))
for f in Path(sys.argv[1]).rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = bench_name(r["Kernel_Name"]) or r["Kernel_Name"][:30]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[k][r["Counter_Name"]] += 1
for k in ("fused_reverse", "fused_apply"):
    c = {n: tot[k][n] / max(cnt[k][n], 1) for n in tot[k]}
    w = c.get("SQ_WAVES", 1)
    print(k, "per wave: VALU %.0f FMA %.0f MUL %.0f ADD %.0f SALU %.0f LDS %.0f  VALU-active/wave %.0f" % tuple(
        c.get(n, 0) / w for n in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_MUL_F32",
                                 "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_VALU")))
PY
done
LIBS="$LIBS" bash tools/ab_lib.sh
