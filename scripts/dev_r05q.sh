bash scripts/dev_ab.sh gpurun_out/r05q "nonl nl4 nl5" "c3:f64 c3:f32" 5
RT_HIP_LIB=cpu-ray-tracing-implementation_amd/build/librt_hip_nl4.so bash scripts/dev_env_ab.sh gpurun_out/r05q "c3:f64 c4:f64" "RT_PARTIAL_BUDGET=8000000000 RT_PARTIAL_BUDGET=2147483648 RT_PARTIAL_BUDGET=1073741824" 3
