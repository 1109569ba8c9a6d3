# Development A/B: bench configs with extra flags / alternative libraries.  bash scripts/dev_ab.sh
set -e
mkdir -p gpurun_out/ab
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --f64-steps 0 "$@" > gpurun_out/ab/$v.json 2>gpurun_out/ab/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));print('$v',d['ms_per_step'], d['config'].get('grid_lanes'), (d.get('parity') or {}).get('rmse'))"
}
run c3 "" --config c3
run c4 "" --config c4 --steps 2 --warmup 1
run c4_g6 "RT_HIP_LIB=$B/librt_hip_g6.so" --config c4 --steps 2 --warmup 1
run c4_g4 "RT_HIP_LIB=$B/librt_hip_g4.so" --config c4 --steps 2 --warmup 1
