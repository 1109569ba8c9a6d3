#!/bin/bash
# GPU box, development: C3 against the wide tree's leaf size and split axes (RT_DEV_WIDE_LEAF / RT_DEV_WIDE_AXES,
# read by the scene compiler at upload)
mkdir -p gpurun_out/r04y
for prec in f32 f64; do
  for leaf in 4 5 6 7 8; do
    RT_DEV_WIDE_LEAF=$leaf timeout -k 10 120 python3 bench.py --config c3 --precision $prec --steps 5 --warmup 1 \
      --no-cpu-baseline --alt-steps 0 > gpurun_out/r04y/c3_${prec}_leaf$leaf.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r04y/c3_${prec}_leaf$leaf.json')); print('c3 $prec leaf $leaf', d['ms_per_step'], round(d['value']/1e3,3))"
  done
done
for prec in f32 f64; do
  for leaf in 6 8; do
    RT_DEV_WIDE_AXES=3 RT_DEV_WIDE_LEAF=$leaf timeout -k 10 120 python3 bench.py --config c3 --precision $prec --steps 5 \
      --warmup 1 --no-cpu-baseline --alt-steps 0 > gpurun_out/r04y/c3_${prec}_ax3_leaf$leaf.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r04y/c3_${prec}_ax3_leaf$leaf.json')); print('c3 $prec axes3 leaf $leaf', d['ms_per_step'], round(d['value']/1e3,3))"
  done
done
