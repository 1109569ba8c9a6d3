# Development A/B: bench configs with extra flags / alternative libraries.  bash scripts/dev_ab.sh
set -e
mkdir -p gpurun_out/ab
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --f64-steps 0 "$@" > gpurun_out/ab/$v.json 2>gpurun_out/ab/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));print('$v',d['ms_per_step'])"
}
run c3 "" --config c3
run c3_prev "RT_HIP_LIB=$B/librt_hip_prev.so" --config c3
run c3b "" --config c3
run c3_prevb "RT_HIP_LIB=$B/librt_hip_prev.so" --config c3
