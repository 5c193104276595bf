#!/bin/bash
# Round 6c: what the per-launch HIP events cost the bench step (unprofiled timed steps first),
# and single-gate cells by XCD block order of reducing launches (QDC_XCD_MAP=3: the reverse
# kernels with their gradient too) — no library change.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r6c
mkdir -p "$OUT"
export TMPDIR=/tmp
QDC_BENCH_UNPROFILED_STEPS=10 timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline \
  --no-gate-sample > "$OUT/bench_unprof.json" 2> "$OUT/bench_unprof.err"
rc=$?; tail -c 200 "$OUT/bench_unprof.json"; [ $rc -eq 0 ] || exit $rc
for x in 1 3 1 3; do
  QDC_XCD_MAP=$x timeout -k 10 300 python -u tools/r5/micro_subset.py --q1 0,12,20,24 \
    --q2 0:1,1:0,5:20,26:27,27:0,1:2,3:9,14:13 > "$OUT/micro_xcd$x.log" 2>&1 || exit $?
  echo "xcd $x"; grep -E 'reverse_q2 |reverse_q1' "$OUT/micro_xcd$x.log" | awk '{print $1,$2,$3,$NF-0, $(NF-3)}' | head -20
done
