#!/bin/bash
# Timing-only ablation builds of the f32 library (QDC_RQ_ABL bits, csrc/qdc_kernels.hpp: 1 no
# stage math, 2 no relayouts, 4 no Gamma, 32 no HBM traffic) into <pkg>/lib-abl<bits>/, next to
# csrc/ so their specialized passes compile from the same headers (the JIT honours the bits:
# the ablation triple is of the kernels that actually run, not the interpreted ones).
set -e
cd "$(dirname "$0")/../.."
PKG=differentiable-quantum-circuit-cuda_amd
FP=$(python3 $PKG/csrc/src_fp.py $PKG/csrc include)
for bits in "$@"; do
  d=$PKG/lib-abl$bits
  mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -fvisibility=hidden \
    -Iinclude -DQDC_SRC_FP=${FP}ull -DQDC_RQ_ABL=$bits -o $d/libqdc_f32.so.tmp $PKG/csrc/qdc.hip -lrccl \
    2> $d/build.log && mv -f $d/libqdc_f32.so.tmp $d/libqdc_f32.so &
done
wait
