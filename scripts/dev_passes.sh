#!/bin/bash
# GPU box, development: ms per frame against the partial-sum budget (render() chunk passes).
#   scripts/dev_passes.sh <outdir> "<config:precision ...>" "<budget bytes ...>" [steps]
set -e
out=$1; runs=$2; budgets=$3; steps=${4:-3}
mkdir -p $out
for r in $runs; do
  cfg=${r%%:*}; prec=${r##*:}
  for b in $budgets; do
    RT_PARTIAL_BUDGET=$b timeout -k 10 600 python3 bench.py --config $cfg --precision $prec --steps $steps --warmup 1 \
      --no-cpu-baseline --alt-steps 0 > $out/${cfg}_${prec}_$b.json 2> $out/${cfg}_${prec}_$b.err
    python3 -c "import json; d=json.load(open('$out/${cfg}_${prec}_$b.json')); print('$cfg $prec budget $b', d['ms_per_step'], 'ms', d['config']['rounds_per_frame'], 'launches')"
  done
done
