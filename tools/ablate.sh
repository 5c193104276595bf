#!/bin/bash
# Build timing-only ablation variants of the f32 library (QDC_RQ_ABL bits, qdc_kernels.hpp) into
# build/abl<bits>/; bench each with QDC_LIB_DIR=build/abl<bits> (results are wrong: timing only,
# QDC_BENCH_ABLATION=1 skips bench.py's sanity checks).
set -e
cd "$(dirname "$0")/.."
for bits in "$@"; do
  d=build/abl$bits
  mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -fvisibility=hidden \
    -Iinclude -DQDC_RQ_ABL=$bits -o $d/libqdc_f32.so differentiable-quantum-circuit-cuda_amd/csrc/qdc.hip -lrccl &
done
wait
