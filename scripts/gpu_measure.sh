#!/bin/bash
# GPU box: the bench line plus rocprofv3 kernel-trace and PMC passes of the given configs.
#   scripts/gpu_measure.sh <tag> "<config> [bench args]" ["<config> [bench args]" ...]
# Output under gpurun_out/<tag>/ (copied back by gpurun); summaries in gpurun_out/<tag>/<cfg>/summary.
# Each GPU step has its own time limit and the chain stops at the first failure.
set -e
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$tag
for spec in "$@"; do
  set -- $spec
  cfg=$1; shift
  timeout -k 10 400 python3 bench.py --config $cfg "$@" > gpurun_out/$tag/bench_$cfg.json 2> gpurun_out/$tag/bench_$cfg.err
  cat gpurun_out/$tag/bench_$cfg.json
  bash scripts/prof_pmc.sh gpurun_out/$tag/$cfg ${tag}_$cfg --config $cfg
done
