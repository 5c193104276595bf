#!/bin/bash
# An experimental build of the f32 library with extra -D switches into <pkg>/lib-<tag>/ (next to
# csrc/, so its specialized passes compile from the same headers with the same switches).
# usage: tools/r5/build_variant.sh <tag> -DNAME=VALUE ...
set -e
cd "$(dirname "$0")/../.."
PKG=differentiable-quantum-circuit-cuda_amd
tag=$1
shift
FP=$(python3 $PKG/csrc/src_fp.py $PKG/csrc include)
d=$PKG/lib-$tag
mkdir -p $d
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -fvisibility=hidden \
  -Iinclude -DQDC_SRC_FP=${FP}ull "$@" -o $d/libqdc_f32.so.tmp $PKG/csrc/qdc.hip -lrccl 2> $d/build.log
mv -f $d/libqdc_f32.so.tmp $d/libqdc_f32.so
