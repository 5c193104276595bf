#!/bin/bash
# Round 5c: (1) the JIT tests (ahead-of-time programs compile nothing; background compiler) and
# the mirror tests; (2) 3 waves/SIMD for the two-state reverse passes (lib-w3: QDC_RW_WAVES=3,
# lib-w3g: + QDC_RQ_GSPLIT=1) against the production library, same box; (3) the shard
# rehearsal with the round-5 library (mirrored sharded sweeps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5c
mkdir -p "$OUT"
export TMPDIR=/tmp
PKG=differentiable-quantum-circuit-cuda_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py tests/test_gpu_mirror.py -x -v -s --timeout 300 \
  --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests.log" | tail -3; [ $rc -eq 0 ] || exit $rc
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], d["value"], "gates/s", d["ms_per_step"], "ms/step", {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01})
PY
}
# variants: base, lib-<tag> builds, and state-layout knobs (interleaved pair off / 1 MiB blocks)
for v in base w3g w3 ilv0 ilv16 base w3g; do
  case $v in
    base) timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $? ;;
    ilv0) QDC_STATE_ILV=0 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $? ;;
    ilv16) QDC_STATE_ILV_BITS=16 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $? ;;
    *) QDC_LIB_DIR=$PWD/$PKG/lib-$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
         --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $? ;;
  esac
  summ "$OUT/b_$v.log" $v
done
TAG=r5c/shard bash tools/shard_rehearsal.sh 2>&1 | tee "$OUT/shard_rehearsal.txt"
