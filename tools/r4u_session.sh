#!/bin/bash
# Why the half-LDS timing probe (scratch/, addresses folded) ran the reverse passes 25 % faster
# than the real half-buffer kernels: one SQ counter pass (instructions, LDS bank conflicts, LDS
# waits) of a short C2 run per library, and the same short run's timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4u}
mkdir -p "$OUT"
export TMPDIR=/tmp
P="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
ABL="QDC_LIB_DIR=$PWD/scratch/lib QDC_SRC_DIR=$PWD/scratch/csrc QDC_BENCH_ABLATION=1"
for v in lib probe; do
  if [ $v = lib ]; then E="QDC_X=0"; else E=$ABL; fi
  env $E timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --layers 4 --no-cpu-baseline --no-gate-sample > "$OUT/t_$v.log" 2>&1 || exit 1
  env $E timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/rq_${v}_p1" -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --layers 4 --no-cpu-baseline --no-gate-sample > "$OUT/sq_$v.log" 2>&1 || exit $?
done
python3 tools/sq_summary.py "$OUT" > "$OUT/sq_summary.txt" 2>&1; head -60 "$OUT/sq_summary.txt"
