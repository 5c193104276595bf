#!/bin/bash
# Round 5d: the packed-FMA forms (QDC_PK_ASM / QDC_PK_VASM / QDC_MATVEC_N): bit-identity of the
# variants' outputs, then the C2 n=28 bench of each, alternating, same box; the sharded GPU
# tests (tiled pack, permuting passes on shards) and the shard rehearsal with them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r5d
mkdir -p "$OUT"
export TMPDIR=/tmp
PKG=differentiable-quantum-circuit-cuda_amd
for v in orig n2asm hyb blt; do
  QDC_LIB_DIR=$PWD/$PKG/lib-$v timeout -k 10 200 python tools/r5/variant_outputs.py "$OUT/out_$v.npz" > "$OUT/out_$v.log" 2>&1 || { cat "$OUT/out_$v.log"; exit 1; }
done
timeout -k 10 200 python tools/r5/variant_outputs.py "$OUT/out_prod.npz" > "$OUT/out_prod.log" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import sys, numpy as np
o = sys.argv[1]
ref = np.load(f"{o}/out_orig.npz")
for v in ("n2asm", "hyb", "blt", "prod"):
    x = np.load(f"{o}/out_{v}.npz")
    print(v, {k: bool(np.array_equal(x[k], ref[k])) for k in ref.files},
          {k: float(np.abs(x[k] - ref[k]).max()) for k in ref.files})
PY
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print(sys.argv[2], d["value"], "gates/s", d["ms_per_step"], "ms/step", {n: (v["launches"], v["avg_ms"]) for n, v in k.items() if v["share"] > 0.01})
PY
}
for v in orig n2asm hyb blt orig hyb blt n2asm; do
  QDC_LIB_DIR=$PWD/$PKG/lib-$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
    --no-cpu-baseline --no-gate-sample > "$OUT/b_$v.log" 2>&1 || exit $?
  summ "$OUT/b_$v.log" $v
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_mirror.py -x -v -s --timeout 300 \
  --timeout-method thread > "$OUT/tests_sharded.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$OUT/tests_sharded.log" | tail -3; [ $rc -eq 0 ] || exit $rc
TAG=r5d/shard bash tools/shard_rehearsal.sh 2>&1 | tee "$OUT/shard_rehearsal.txt"
