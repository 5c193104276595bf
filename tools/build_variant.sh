#!/bin/bash
# Build the f32 library with extra compile-time defines into build/<name>/ (A/B experiments):
#   bash tools/build_variant.sh <name> -DQDC_RQ_GSPLIT=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/$name
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -fvisibility=hidden \
  -Iinclude "$@" -o build/$name/libqdc_f32.so differentiable-quantum-circuit-cuda_amd/csrc/qdc.hip -lrccl
