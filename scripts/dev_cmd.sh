set -e
mkdir -p gpurun_out/s15
B=cpu-ray-tracing-implementation_amd/build
run() {  # tag lib config precision
  L=""; [ $2 != base ] && L="RT_HIP_LIB=$B/librt_hip_$2.so"
  env $L timeout -k 10 200 python3 bench.py --config $3 --precision $4 --steps 10 --no-cpu-baseline --alt-steps 0 > gpurun_out/s15/$1.json 2>gpurun_out/s15/$1.err
  python3 -c "import json;d=json.load(open('gpurun_out/s15/$1.json'));print('$1',d['ms_per_step'], d['value'])"
}
run c2_f64_fw5 fw5 c2 f64
run c2_f64_fw3 fw3 c2 f64
run c2_f64_base base c2 f64
run c4_f32_gw5 gw5 c4 f32
run c4_f32_base base c4 f32
