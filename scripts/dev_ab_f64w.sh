# Development A/B of the fp64 wide kernels' wave budgets (a: LDS 4 / HBM 5, b: LDS 2 / HBM 3; default
# LDS none / HBM 4) on C3 / C4 fp64.
set -e
mkdir -p gpurun_out/ab64w
B=cpu-ray-tracing-implementation_amd/build
run() {  # name, env, args
  local v=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --no-cpu-baseline --alt-steps 0 "$@" > gpurun_out/ab64w/$v.json 2>gpurun_out/ab64w/$v.err
  python3 -c "import json;d=json.load(open('gpurun_out/ab64w/$v.json'));print('$v',d['ms_per_step'], d['value'], d['config'].get('grid_lanes'), d['config']['segments_per_sample'])"
}
for v in "" a b; do
  e=""; [ -n "$v" ] && e="RT_HIP_LIB=$B/librt_hip_$v.so"
  run c3_f64_${v:-base} "$e" --config c3 --precision f64 --steps 3
  run c4_f64_${v:-base} "$e" --config c4 --precision f64 --steps 2
done
