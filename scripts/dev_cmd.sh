set -e
mkdir -p gpurun_out/s9
B=cpu-ray-tracing-implementation_amd/build
run() {  # tag lib config precision
  L=""; [ $2 != base ] && L="RT_HIP_LIB=$B/librt_hip_$2.so"
  env $L timeout -k 10 200 python3 bench.py --config $3 --precision $4 --steps 10 --no-cpu-baseline --alt-steps 0 > gpurun_out/s9/$1.json 2>gpurun_out/s9/$1.err
  python3 -c "import json;d=json.load(open('gpurun_out/s9/$1.json'));print('$1',d['ms_per_step'], d['value'])"
}
run c2_f64_new base c2 f64
run c2_f64_prev prev c2 f64
run c2_f32_new base c2 f32
run c2_f32_prev prev c2 f32
run c3_w8 w8 c3 f32
run c3_w6 w6 c3 f32
run c3_sb56 sb56 c3 f32
run c3_prev prev c3 f32
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s9/tests.log 2>&1
tail -1 gpurun_out/s9/tests.log
