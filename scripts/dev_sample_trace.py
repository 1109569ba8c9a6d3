"""Dev tool: per-sample, per-depth comparison of one pixel (fp32 / fp64 device vs oracle).

  python scripts/dev_sample_trace.py SCENE WIDTH ASPECT SPP DEPTH X Y            # find the divergent sample
  python scripts/dev_sample_trace.py SCENE WIDTH ASPECT SPP DEPTH X Y S          # segment trace of sample S:
      device lines ("[dev]") need `make trace` (build/librt_hip_trace.so), oracle lines ("[trace]") go to stderr
"""
import os, sys, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO + '/cpu-ray-tracing-implementation_amd/python'); sys.path.insert(0, REPO + '/oracle')
import rt_amd, oracle
from rt_amd import scenes, abi
name, w, a, spp, depth, x, y = sys.argv[1], int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7])
trace = len(sys.argv) > 8
if trace:
    abi.lib_path = lambda: os.path.join(abi.BUILD_DIR, 'librt_hip_trace.so')
ctx = rt_amd.Context(0)
desc, cam, _, _ = scenes.SCENES[name](width=w, aspect=a)
ctx.upload(desc)
osc = oracle.from_desc(desc)
tile = [(x, y, 1, 1)]
if trace:
    s = int(sys.argv[8])
    for prec in (abi.RT_PREC_F32, abi.RT_PREC_F64):
        print(f'--- device precision {prec}', flush=True)
        v = ctx.render(cam, 1, depth, seed=7, precision=prec, tiles=tile, first_sample=s)[0]
        print('value', v, flush=True)
    print('--- oracle', flush=True)
    oracle.lib().orc_set_trace(1)
    print('value', oracle.render(osc, cam, 1, depth, seed=7, threads=1, tiles=tile, first_sample=s)[0][0], flush=True)
    sys.exit(0)
for s in range(spp):
    for d in range(1, depth + 1):
        f32 = ctx.render(cam, 1, d, seed=7, precision=abi.RT_PREC_F32, tiles=tile, first_sample=s)[0]
        f64 = ctx.render(cam, 1, d, seed=7, precision=abi.RT_PREC_F64, tiles=tile, first_sample=s)[0]
        ref = oracle.render(osc, cam, 1, d, seed=7, tiles=tile, first_sample=s)[0][0]
        flag = '  <-- DIVERGES' if np.abs(f32 - ref).max() > 1e-3 else ''
        print(f"sample {s} depth {d}: f32={f32} f64={f64} ref={ref}{flag}", flush=True)
