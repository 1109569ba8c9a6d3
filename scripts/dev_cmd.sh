set -e
mkdir -p gpurun_out/s14
for c in "c2 f64" "c2 f32" "c3 f32" "c3 f64" "c4 f32" "c5 f32"; do
  timeout -k 10 150 python3 scripts/dev_wide_stats.py $c >> gpurun_out/s14/stats.txt 2>&1
done
grep -v amdgpu.ids gpurun_out/s14/stats.txt
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s14/smoke.log 2>&1
tail -n 1 gpurun_out/s14/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/s14/bench_default.json 2> gpurun_out/s14/bench_default.err
cut -c1-300 gpurun_out/s14/bench_default.json
