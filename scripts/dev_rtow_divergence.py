"""Dev tool: fp32 vs oracle divergence on RTOW (the specular-chain scene) for one or more builds.
    python scripts/dev_rtow_divergence.py [lib.so ...]   (names under the build directory)"""
import os, sys, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO + '/cpu-ray-tracing-implementation_amd/python'); sys.path.insert(0, REPO + '/oracle')
import rt_amd, oracle
from rt_amd import scenes, abi
cases = [('rtow', 96, 64), ('rtow', 48, 512)]
refs = {}
for name, w, spp in cases:
    desc, cam, _, _ = scenes.SCENES[name](width=w, aspect=1.5)
    refs[(name, w, spp)] = (desc, cam, oracle.render(oracle.from_desc(desc), cam, spp, 50, seed=7, threads=16)[0])
for lib in (sys.argv[1:] or ['librt_hip.so']):
    abi.lib_path = lambda lib=lib: os.path.join(abi.BUILD_DIR, lib)
    abi._lib = None
    ctx = rt_amd.Context(0)
    for (name, w, spp), (desc, cam, ref) in refs.items():
        ctx.upload(desc)
        img = ctx.render(cam, spp, 50, seed=7, precision=abi.RT_PREC_F32).astype(np.float64)
        d = np.abs(img - ref).max(-1)
        rmse = np.sqrt(((img - ref) ** 2).reshape(-1, 3).mean(0))
        print(f"{lib} {name} {w}px spp={spp}: rmse={rmse} n>1e-3={int((d > 1e-3).sum())} n>1e-4={int((d > 1e-4).sum())}/{d.size}", flush=True)
    ctx.close()
