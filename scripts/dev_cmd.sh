set -e
mkdir -p gpurun_out/r03s
bash scripts/gpu_measure.sh r03s "c4 f64" "c4 f32" "c5 f64" "c5 f32" -- c4 c5
