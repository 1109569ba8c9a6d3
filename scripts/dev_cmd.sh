set -e
mkdir -p gpurun_out/s17
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "no_light or fp64_device or fp32_device" > gpurun_out/s17/tests.log 2>&1 || (tail -30 gpurun_out/s17/tests.log; exit 1)
tail -1 gpurun_out/s17/tests.log
