#!/bin/bash
# GPU box: the round's measurements. For every "<config> <precision>" spec: kernel trace + PMC passes
# (scripts/prof_pmc.sh) whose summaries are copied into profiles/ on the box; then one bench line per
# config (fp64 headline + fp32 alt line, CPU baseline and full-size parity rows), which reads those
# summaries for its rooflines.
#   scripts/gpu_measure.sh <tag> "<config> <precision>" ... -- <config> ...
# Output under gpurun_out/<tag>/ (copied back by gpurun). Each GPU step has its own time limit and
# the chain stops at the first failure.
set -e
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/$tag profiles
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  set -- $1 "${@:2}"
  cfg=$1; prec=$2; shift 2
  bash scripts/prof_pmc.sh gpurun_out/$tag/${cfg}_$prec ${tag}_${cfg}_$prec --config $cfg --precision $prec
  cp gpurun_out/$tag/${cfg}_$prec/summary/* profiles/
done
[ "$1" == "--" ] && shift
for cfg in "$@"; do
  timeout -k 10 600 python3 bench.py --config $cfg > gpurun_out/$tag/bench_$cfg.json 2> gpurun_out/$tag/bench_$cfg.err
  cut -c1-400 gpurun_out/$tag/bench_$cfg.json
done
