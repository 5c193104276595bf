#!/bin/bash
# Round 5h: gate-shaped streaming patterns (stream_probe rows), then same-box C2 A/B: wave
# stagger (lib-stag2 / lib-stag4: QDC_RW_STAGGER), longer tile rows (QDC_FUSE_LCMIN /
# QDC_RQ_PERM_LOW), against the production library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5h
mkdir -p "$OUT"
export TMPDIR=/tmp
PKG=differentiable-quantum-circuit-cuda_amd
timeout -k 10 120 tools/bin/stream_probe > "$OUT/stream_probe.txt" 2>&1 || exit $?
grep rows "$OUT/stream_probe.txt"
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], d["value"], "gates/s", d["ms_per_step"], "ms/step", {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01})
PY
}
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample"
for v in base stag2 stag4 lc4p5 p5 lc4p6 base stag4; do
  case $v in
    base) timeout -k 10 300 $B > "$OUT/b_$v.log" 2>&1 || exit $? ;;
    lc4p5) QDC_FUSE_LCMIN=4 QDC_RQ_PERM_LOW=5 timeout -k 10 300 $B > "$OUT/b_$v.log" 2>&1 || exit $? ;;
    lc4p6) QDC_FUSE_LCMIN=4 QDC_RQ_PERM_LOW=6 timeout -k 10 300 $B > "$OUT/b_$v.log" 2>&1 || exit $? ;;
    p5) QDC_RQ_PERM_LOW=5 timeout -k 10 300 $B > "$OUT/b_$v.log" 2>&1 || exit $? ;;
    *) QDC_LIB_DIR=$PWD/$PKG/lib-$v timeout -k 10 300 $B > "$OUT/b_$v.log" 2>&1 || exit $? ;;
  esac
  summ "$OUT/b_$v.log" $v
done
