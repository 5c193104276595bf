#!/bin/bash
# Timing-only probe: one-wave passes with half the LDS relayout buffer (scratch/ build,
# -DQDC_ABL_BUFDIV=2: wrong results, the same instruction stream; 8 KiB instead of 16 KiB per
# wave, so up to 5 waves per SIMD) against the committed library, with the persistent grid sized
# for the higher occupancy (QDC_FUSED_BLOCKS) or not.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4p}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gate-sample > "$OUT/b_$tag.log" 2>&1 || return 1
  python3 -c "
import json
d=json.loads([l for l in open('$OUT/b_$tag.log') if l.startswith('{')][-1])
print('$tag', d['value'], {k:(v['launches'],v['avg_ms']) for k,v in d['kernels'].items() if v['share']>0.01})"
}
ABL="QDC_LIB_DIR=$PWD/scratch/lib QDC_SRC_DIR=$PWD/scratch/csrc QDC_BENCH_ABLATION=1"
for r in 1 2; do
  run base_$r QDC_X=0 || exit 1
  run base_fb5120_$r QDC_FUSED_BLOCKS=5120 || exit 1
  run half_$r $ABL || exit 1
  run half_fb5120_$r $ABL QDC_FUSED_BLOCKS=5120 || exit 1
done
