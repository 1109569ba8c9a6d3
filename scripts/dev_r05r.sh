bash scripts/dev_ab.sh gpurun_out/r05r "t0 t5 t21 t21s22" "c4:f32 c4:f64" 3
RT_HIP_LIB=cpu-ray-tracing-implementation_amd/build/librt_hip_t21s22.so timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_wide.py -k "not multi" 2>&1 | tail -3
