# Development A/B: bench configs with extra flags / alternative libraries.  bash scripts/dev_ab.sh
set -e
mkdir -p gpurun_out/ab
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --f64-steps 0 "$@" > gpurun_out/ab/$v.json 2>gpurun_out/ab/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));print('$v',d['ms_per_step'], d['config'].get('grid_lanes'), (d.get('parity') or {}).get('rmse'))"
}
for i in 1 2; do
run c2_base$i "" --config c2 --steps 20
run c2_w8_$i "RT_HIP_LIB=$B/librt_hip_w8.so" --config c2 --steps 20
run c2_w8cb0_$i "RT_HIP_LIB=$B/librt_hip_w8cb0.so" --config c2 --steps 20
run c2_cb0_$i "RT_HIP_LIB=$B/librt_hip_cb0.so" --config c2 --steps 20
done
