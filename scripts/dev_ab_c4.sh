# Development A/B of trace_wide code shapes on C4 / C3 fp32 (v0: all round-3 switches off; v1: child by
# masks; v2: clamped pop; v3: branch-free push; v4: triangle words prefetched; v5: triangle+quad kernel).
#   bash scripts/dev_ab_c4.sh v0 v1 ...
set -e
mkdir -p gpurun_out/abc4
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --alt-steps 0 "$@" > gpurun_out/abc4/$v.json 2>gpurun_out/abc4/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/abc4/$v.json'));print('$v',d['ms_per_step'], d['value'], d['config'].get('grid_lanes'), d['config']['segments_per_sample'])"
}
for v in "$@"; do
  run c4_$v "RT_HIP_LIB=$B/librt_hip_$v.so" --config c4 --precision f32 --steps 3
  run c3_$v "RT_HIP_LIB=$B/librt_hip_$v.so" --config c3 --precision f32 --steps 5
done
