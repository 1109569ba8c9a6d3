#!/bin/bash
# Development: registers, scratch and occupancy of one kernel family without a full build.
#   scripts/dev_usage.sh <1 flat | 2 wide | 3 linear> [-DFOO=1 ...]
set -e
cd "$(dirname "$0")/.."
only=$1; shift
log=$(mktemp /tmp/usage.XXXX.log)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -ffp-contract=on -fno-slp-vectorize --offload-arch=gfx950 --cuda-device-only \
  -Rpass-analysis=kernel-resource-usage -DRT_DEV_ONLY=$only "$@" -c -o /dev/null \
  cpu-ray-tracing-implementation_amd/csrc/rt_kernels.hip 2> $log
python3 scripts/kernel_usage.py $log k_persist_occ
