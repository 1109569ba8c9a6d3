#!/bin/bash
# Development: build librt_hip.so with extra -D flags under another name, for A/B runs
# (RT_HIP_LIB=<path> python bench.py ...).   scripts/build_variant.sh <name> -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=cpu-ray-tracing-implementation_amd/build/librt_hip_$name.so
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -ffp-contract=on -fno-slp-vectorize --offload-arch=gfx950 "$@" -shared -o $out \
  cpu-ray-tracing-implementation_amd/csrc/rt_kernels.hip cpu-ray-tracing-implementation_amd/csrc/rt_multi.hip \
  cpu-ray-tracing-implementation_amd/csrc/scene_compile.cpp -ldl
echo $out
