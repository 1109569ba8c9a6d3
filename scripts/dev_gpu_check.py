import os, sys, time, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO + '/cpu-ray-tracing-implementation_amd/python'); sys.path.insert(0, REPO + '/oracle')
import rt_amd, oracle
from rt_amd import scenes, abi
ctx = rt_amd.Context(0)
for name, w, spp, depth in [('cornell_box', 64, 16, 8), ('cornell_box_with_volume', 64, 8, 5), ('three_material_ball', 64, 8, 5), ('rtow', 60, 8, 50)]:
    desc, cam, _, _ = scenes.SCENES[name](width=w)
    ctx.upload(desc)
    osc = oracle.from_desc(desc)
    ref, segs = oracle.render(osc, cam, spp, depth, seed=7)
    for prec in (abi.RT_PREC_F64, abi.RT_PREC_F32):
        t0 = time.time()
        img = ctx.render(cam, spp, depth, seed=7, precision=prec)
        dt = time.time() - t0
        st = ctx.stats()
        d = np.abs(img - ref)
        rmse = np.sqrt(((img - ref) ** 2).reshape(-1, 3).mean(0))
        print(f"{name:26s} prec={prec} max|d|={d.max():.3e} rmse={rmse} frac>1e-3={np.mean(d.max(-1) > 1e-3):.4f} segs gpu/orc={st.segments}/{segs} it={st.iterations} {dt*1e3:.1f}ms", flush=True)
    ctx.reset_counters()
