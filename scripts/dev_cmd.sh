set -e
mkdir -p gpurun_out/s13
run() {  # tag env config precision
  env $2 timeout -k 10 200 python3 bench.py --config $3 --precision $4 --steps 10 --no-cpu-baseline --alt-steps 0 > gpurun_out/s13/$1.json 2>gpurun_out/s13/$1.err
  python3 -c "import json;d=json.load(open('gpurun_out/s13/$1.json'));print('$1',d['ms_per_step'], d['value'])"
}
run c3_f32 "" c3 f32
run c3_f64 "" c3 f64
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s13/tests.log 2>&1
tail -1 gpurun_out/s13/tests.log
