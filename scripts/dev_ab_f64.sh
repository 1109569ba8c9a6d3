# Development A/B of the fp64 C2 kernel: cold path state in LDS (c4: 4 waves, c5: 5 waves), the fp32
# item layout with tail items (t4), both (ct4), against the default build.   bash scripts/dev_ab_f64.sh
set -e
mkdir -p gpurun_out/ab64
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --alt-steps 0 "$@" > gpurun_out/ab64/$v.json 2>gpurun_out/ab64/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab64/$v.json'));print('$v',d['ms_per_step'], d['value'], d['config'].get('grid_lanes'), d['config']['segments_per_sample'])"
}
run f64_base "" --config c2 --precision f64 --steps 10
for v in c4 c5 t4 ct4; do run f64_$v "RT_HIP_LIB=$B/librt_hip_$v.so" --config c2 --precision f64 --steps 10; done
run f64_base2 "" --config c2 --precision f64 --steps 10
