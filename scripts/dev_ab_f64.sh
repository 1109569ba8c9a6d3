# Development A/B of the fp64 C2 kernel (flat program at 4 / 5 waves per SIMD, and the ordered
# linear program), then the fp32 C2 line for regressions.   bash scripts/dev_ab_f64.sh
set -e
mkdir -p gpurun_out/ab64
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --alt-steps 0 "$@" > gpurun_out/ab64/$v.json 2>gpurun_out/ab64/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab64/$v.json'));print('$v',d['ms_per_step'], d['value'], d['config'].get('grid_lanes'), d['config']['segments_per_sample'])"
}
run f64_w4 "" --config c2 --precision f64 --steps 5
run f64_w5 "RT_HIP_LIB=$B/librt_hip_f64w5.so" --config c2 --precision f64 --steps 5
run f64_ordered "" --config c2 --precision f64 --steps 3 --traversal ordered
run f32 "" --config c2 --precision f32 --steps 20
