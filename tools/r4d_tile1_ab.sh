#!/bin/bash
# One-state (forward) passes on 2^11-amplitude one-wave tiles with five register slots
# (QDC_TILE1_CHUNKS=1024, QDC_RW bit 1; bit 3: prefetching) against the default 2^12 four-wave
# tiles: parity of the fused tests in the new configuration, then an interleaved C2 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r4d
for rw in 3 11; do
  QDC_TILE1_CHUNKS=1024 QDC_RW=$rw timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_circuit.py \
    -k "not ablation" -x -q --timeout 300 --timeout-method thread > gpurun_out/r4d/tests_t1k_rw$rw.log 2>&1
  rc=$?; tail -2 gpurun_out/r4d/tests_t1k_rw$rw.log; [ $rc -eq 0 ] || exit $rc
done
TAG=r4d REPS=2 STEPS_N=5 CFGS="- QDC_TILE1_CHUNKS=1024,QDC_RW=3 QDC_TILE1_CHUNKS=1024,QDC_RW=11 QDC_SPEC_FWD=0 QDC_TILE1_CHUNKS=1024,QDC_RW=11,QDC_SPEC_FWD=0" bash tools/ab_env.sh
