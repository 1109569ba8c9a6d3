# Development: frame times of the current build on every config in both precisions.
set -e
mkdir -p gpurun_out/now
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --alt-steps 0 "$@" > gpurun_out/now/$v.json 2>gpurun_out/now/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/now/$v.json'));print('$v',d['ms_per_step'], d['value'], d['config'].get('grid_lanes'), d['config']['segments_per_sample'])"
}
run c3_f64 "" --config c3 --precision f64 --steps 3
run c4_f64 "" --config c4 --precision f64 --steps 2
run c2_f64 "" --config c2 --precision f64 --steps 10
run c3_f32 "" --config c3 --precision f32 --steps 5
run c4_f32 "" --config c4 --precision f32 --steps 3
