# Development A/B on C4 fp32: pause thresholds 40 / 56 (default 48) and 22 LDS stack entries at 7 waves.
set -e
mkdir -p gpurun_out/abc4
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --alt-steps 0 "$@" > gpurun_out/abc4/$v.json 2>gpurun_out/abc4/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/abc4/$v.json'));print('$v',d['ms_per_step'], d['value'], d['config'].get('grid_lanes'), d['config']['segments_per_sample'])"
}
run c4_base "" --config c4 --precision f32 --steps 3
for v in p40 p56 s22; do run c4_$v "RT_HIP_LIB=$B/librt_hip_$v.so" --config c4 --precision f32 --steps 3; done
run c5_f64 "" --config c5 --precision f64 --steps 2
