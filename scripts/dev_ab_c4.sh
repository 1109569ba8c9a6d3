# Development A/B of the C4 kernel's tree in HBM: quantised 4-wide nodes (default), float 4-wide
# (RT_DEV_WIDEQ=0), compressed 8-wide (RT_DEV_WIDEQ=8); leaves of 3 / 4 triangles.   bash scripts/dev_ab_c4.sh
set -e
mkdir -p gpurun_out/abc4
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --alt-steps 0 "$@" > gpurun_out/abc4/$v.json 2>gpurun_out/abc4/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/abc4/$v.json'));print('$v',d['ms_per_step'], d['value'], d['config'].get('grid_lanes'), d['config']['segments_per_sample'])"
}
run c4_q4 "" --config c4 --precision f32 --steps 3
run c4_f4 "RT_DEV_WIDEQ=0" --config c4 --precision f32 --steps 3
run c4_q4_leaf3 "RT_DEV_WIDE_LEAF=3" --config c4 --precision f32 --steps 3
run c4_f4_leaf3 "RT_DEV_WIDEQ=0 RT_DEV_WIDE_LEAF=3" --config c4 --precision f32 --steps 3
run c4_q8 "RT_DEV_WIDEQ=8" --config c4 --precision f32 --steps 3
