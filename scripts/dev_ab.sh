# Development A/B: bench configs with extra flags / alternative libraries.  bash scripts/dev_ab.sh
set -e
mkdir -p gpurun_out/ab
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline --f64-steps 0 "$@" > gpurun_out/ab/$v.json 2>gpurun_out/ab/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab/$v.json'));print('$v',d['ms_per_step'])"
}
run c3_leaf6 "RT_DEV_WIDE_LEAF=6" --config c3
run c3_leaf7 "RT_DEV_WIDE_LEAF=7" --config c3
run c3_l6ct8 "RT_DEV_WIDE_LEAF=6 RT_DEV_WIDE_CT=8" --config c3
run c3_l5ct8 "RT_DEV_WIDE_LEAF=5 RT_DEV_WIDE_CT=8" --config c3
run c3_l4ct8 "RT_DEV_WIDE_LEAF=4 RT_DEV_WIDE_CT=8" --config c3
run c4_leaf4 "" --config c4 --steps 2 --warmup 1
run c4_leaf6 "RT_DEV_WIDE_LEAF=6" --config c4 --steps 2 --warmup 1
