#!/bin/bash
# GPU box, development: ms per frame of one config under different environment settings of the library.
#   scripts/dev_env_ab.sh <outdir> "<config:precision ...>" "<NAME=value[,NAME=value] ...>" [steps]
# ("-" runs without extra settings)
set -e
out=$1; runs=$2; envs=$3; steps=${4:-3}
mkdir -p $out
for r in $runs; do
  cfg=${r%%:*}; prec=${r##*:}
  for e in $envs; do
    tag=$(echo "$e" | tr ',=' '__')
    ev=""; [ "$e" != "-" ] && ev=$(echo "$e" | tr ',' ' ')
    env $ev timeout -k 10 600 python3 bench.py --config $cfg --precision $prec --steps $steps --warmup 1 \
      --no-cpu-baseline --alt-steps 0 > $out/${cfg}_${prec}_$tag.json 2> $out/${cfg}_${prec}_$tag.err
    python3 -c "import json; d=json.load(open('$out/${cfg}_${prec}_$tag.json')); print('$cfg $prec $e', d['ms_per_step'], 'ms', d['config']['rounds_per_frame'], 'launches')"
  done
done
