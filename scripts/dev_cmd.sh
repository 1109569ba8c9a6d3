set -e
mkdir -p gpurun_out/s11
B=cpu-ray-tracing-implementation_amd/build
run() {  # tag lib config precision
  L=""; [ $2 != base ] && L="RT_HIP_LIB=$B/librt_hip_$2.so"
  env $L timeout -k 10 200 python3 bench.py --config $3 --precision $4 --steps 5 --no-cpu-baseline --alt-steps 0 > gpurun_out/s11/$1.json 2>gpurun_out/s11/$1.err
  python3 -c "import json;d=json.load(open('gpurun_out/s11/$1.json'));print('$1',d['ms_per_step'], d['value'])"
}
for v in sb40 sb44 base; do run c3_f32_$v $v c3 f32; done
for v in gsb40 gsb56 base; do run c4_f32_$v $v c4 f32; done
for v in gsb40 base; do run c4_f64_$v $v c4 f64; done
