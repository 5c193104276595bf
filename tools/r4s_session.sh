#!/bin/bash
# Occupancy variants of the half-buffer kernels (builds under scratch*/, headers beside them):
# two-state reverse passes compiled for 3 waves per SIMD (scratch3), and one-state forward passes
# for 5 (scratch4, with the reverse at 3), against the committed library; C2 A/B, 2 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4s}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for v in lib scratch3 scratch4; do
    if [ $v = lib ]; then E=""; else E="QDC_LIB_DIR=$PWD/$v/lib QDC_SRC_DIR=$PWD/$v/csrc"; fi
    env $E timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/b_${v}_$r.log" 2>&1 || { tail -5 "$OUT/b_${v}_$r.log"; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('$OUT/b_${v}_$r.log') if l.startswith('{')][-1])
print('$v', d['value'], {k:(v['launches'],v['avg_ms']) for k,v in d['kernels'].items() if v['share']>0.01})"
  done
done
