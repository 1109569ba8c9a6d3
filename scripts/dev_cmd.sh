set -e
mkdir -p gpurun_out/s18
B=cpu-ray-tracing-implementation_amd/build
run() {  # tag lib config precision
  L=""; [ $2 != base ] && L="RT_HIP_LIB=$B/librt_hip_$2.so"
  env $L timeout -k 10 200 python3 bench.py --config $3 --precision $4 --steps 10 --no-cpu-baseline --alt-steps 0 > gpurun_out/s18/$1.json 2>gpurun_out/s18/$1.err
  python3 -c "import json;d=json.load(open('gpurun_out/s18/$1.json'));print('$1',d['ms_per_step'], d['value'])"
}
run c2_f64_cmp cmp64 c2 f64
run c2_f64_base base c2 f64
run c2_f64_cmp2 cmp64 c2 f64
run c2_f64_base2 base c2 f64
