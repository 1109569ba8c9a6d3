# Development A/B of the fp64 BVH / linear kernels' wave budgets (w3, w4) on C3, C4, C5 fp64.
set -e
mkdir -p gpurun_out/ab64c
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --alt-steps 0 "$@" > gpurun_out/ab64c/$v.json 2>gpurun_out/ab64c/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab64c/$v.json'));print('$v',d['ms_per_step'], d['value'], d['config'].get('grid_lanes'), d['config']['segments_per_sample'])"
}
for v in "" w3 w4; do
  e=""; [ -n "$v" ] && e="RT_HIP_LIB=$B/librt_hip_$v.so"
  run c3_f64_${v:-base} "$e" --config c3 --precision f64 --steps 3
  run c5_f64_${v:-base} "$e" --config c5 --precision f64 --steps 1
  run c4_f64_${v:-base} "$e" --config c4 --precision f64 --steps 1
done
