set -e
mkdir -p gpurun_out/s6
run() {  # tag env config precision
  env $2 timeout -k 10 200 python3 bench.py --config $3 --precision $4 --steps 5 --no-cpu-baseline --alt-steps 0 > gpurun_out/s6/$1.json 2>gpurun_out/s6/$1.err
  python3 -c "import json;d=json.load(open('gpurun_out/s6/$1.json'));print('$1',d['ms_per_step'], d['value'])"
}
run c4_f32 "" c4 f32
run c4_f64 "" c4 f64
run c3_f32 "" c3 f32
run c3_f64 "" c3 f64
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s6/tests.log 2>&1
tail -2 gpurun_out/s6/tests.log
