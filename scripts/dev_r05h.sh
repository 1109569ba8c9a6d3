mkdir -p gpurun_out/r05h
for r in c4:f64 c4:f32 c3:f64 c3:f32; do cfg=${r%%:*}; prec=${r##*:};
 (cd tmp_r04 && timeout -k 10 300 python3 bench.py --config $cfg --precision $prec --steps 3 --warmup 1 --no-cpu-baseline --alt-steps 0 > ../gpurun_out/r05h/r04_${cfg}_${prec}.json 2> ../gpurun_out/r05h/r04_${cfg}_${prec}.err) || exit 1
 python3 -c "import json; d=json.load(open('gpurun_out/r05h/r04_${cfg}_${prec}.json')); print('r04 $cfg $prec', d['ms_per_step'])"
done
bash scripts/dev_ab.sh gpurun_out/r05h "wm0nl wm0l5" "c4:f64 c4:f32 c3:f64 c3:f32" 3
