#!/bin/bash
# GPU box, development: C1 (a small frame) against the work-item size -- explicit --chunk values, and the
# automatic size under RT_ITEMS_TARGET (items the frame should have at least; rt_kernels.hip render())
mkdir -p gpurun_out/r04x
run() {  # <tag> <precision> [bench args...]
  local tag=$1 prec=$2; shift 2
  timeout -k 10 120 python3 bench.py --config c1 --precision $prec --steps 20 --warmup 2 --no-cpu-baseline \
    --alt-steps 0 "$@" > gpurun_out/r04x/c1_${prec}_${tag}.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r04x/c1_${prec}_${tag}.json')); print('c1 $prec $tag', d['ms_per_step'], round(d['value']/1e3,3))"
}
for prec in f64 f32; do
  for ch in 2 4 8; do run chunk$ch $prec --chunk $ch; done
  for t in 0 1000000 2500000 5000000; do RT_ITEMS_TARGET=$t run target$t $prec; done
done
