#!/bin/bash
# GPU box, development A/B: ms per frame of library variants (scripts/build_variant.sh) on bench configs.
#   scripts/dev_ab.sh <outdir> "<variant ...>" "<config:precision ...>" [steps]
# variant "base" is the default librt_hip.so. Prints one line per run; the JSON lines go to <outdir>.
set -e
out=$1; variants=$2; runs=$3; steps=${4:-5}
mkdir -p $out
B=cpu-ray-tracing-implementation_amd/build
for r in $runs; do
  cfg=${r%%:*}; prec=${r##*:}
  for v in $variants; do
    lib=""
    [ "$v" != base ] && lib=$B/librt_hip_$v.so
    RT_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg --precision $prec --steps $steps --warmup 1 \
      --no-cpu-baseline --alt-steps 0 > $out/${v}_${cfg}_${prec}.json 2> $out/${v}_${cfg}_${prec}.err
    python3 -c "import json,sys; d=json.load(open('$out/${v}_${cfg}_${prec}.json')); print('$v $cfg $prec', d['ms_per_step'], 'ms', round(d['value']/1e3, 3), 'Gsamples/s')"
  done
done
