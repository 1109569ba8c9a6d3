set -e
mkdir -p gpurun_out/final
timeout -k 10 300 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
tail -1 gpurun_out/final/gpu_tests.log
