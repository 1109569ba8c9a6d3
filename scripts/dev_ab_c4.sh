# Development A/B of the C4 kernel: LDS stack entries / waves per SIMD (s22w7, s20w8) against the
# default (24 entries, 6 waves).   bash scripts/dev_ab_c4.sh
set -e
mkdir -p gpurun_out/abc4
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --alt-steps 0 "$@" > gpurun_out/abc4/$v.json 2>gpurun_out/abc4/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/abc4/$v.json'));print('$v',d['ms_per_step'], d['value'], d['config'].get('grid_lanes'), d['config']['segments_per_sample'])"
}
run c4_base "" --config c4 --precision f32 --steps 3
run c4_s22w7 "RT_HIP_LIB=$B/librt_hip_s22w7.so" --config c4 --precision f32 --steps 3
run c4_s20w8 "RT_HIP_LIB=$B/librt_hip_s20w8.so" --config c4 --precision f32 --steps 3
