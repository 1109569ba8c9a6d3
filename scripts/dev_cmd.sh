set -e
mkdir -p gpurun_out/scal
timeout -k 10 200 python3 scripts/dev_scaling.py --config c2 --precision f64 > gpurun_out/scal/c2_f64.log 2>&1
timeout -k 10 200 python3 scripts/dev_scaling.py --config c2 > gpurun_out/scal/c2.log 2>&1
timeout -k 10 200 python3 scripts/dev_scaling.py --config c3 > gpurun_out/scal/c3.log 2>&1
grep world gpurun_out/scal/*.log | cut -c1-220
