set -e
mkdir -p gpurun_out/s4
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s4/tests.log 2>&1
tail -2 gpurun_out/s4/tests.log
B=cpu-ray-tracing-implementation_amd/build
run() {  # tag lib config precision
  L=""; [ $2 != base ] && L="RT_HIP_LIB=$B/librt_hip_$2.so"
  env $L timeout -k 10 200 python3 bench.py --config $3 --precision $4 --steps 10 --no-cpu-baseline --alt-steps 0 > gpurun_out/s4/$1.json 2>gpurun_out/s4/$1.err
  python3 -c "import json;d=json.load(open('gpurun_out/s4/$1.json'));print('$1',d['ms_per_step'], d['value'])"
}
run c2_f64 base c2 f64
run c2_f32 base c2 f32
run c5_f64 base c5 f64
run c5_f32 base c5 f32
run c3_f32 base c3 f32
run c3_f64 base c3 f64
run c4_f32 base c4 f32
