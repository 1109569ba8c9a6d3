#!/usr/bin/env python3
"""Development: render one tile of a config (e.g. a single slow pixel) and print the host time.
    python scripts/dev_pixel.py --config c4 --precision f64 --tile 1043,829,1,1 [--spp N]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))
import rt_amd  # noqa: E402
from rt_amd import abi, plugin  # noqa: E402
from bench import CONFIGS, sponza_asset  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--precision", default="f64")
ap.add_argument("--tile", default="1043,829,1,1")
ap.add_argument("--spp", type=int, default=0)
a = ap.parse_args()
scene, width, aspect, spp, depth = CONFIGS[a.config]
if scene == "sponza":
    sponza_asset()
cs = plugin.ConfigScene(scene, width, aspect)
ctx = rt_amd.Context(0)
ctx.upload(cs.desc)
prec = abi.RT_PREC_F64 if a.precision == "f64" else abi.RT_PREC_F32
t = tuple(int(x) for x in a.tile.split(","))
for _ in range(2):
    t0 = time.perf_counter()
    img = ctx.render(cs.cam, a.spp or spp, depth, seed=1, precision=prec, tiles=[t])
    print(f"tile {t}: {(time.perf_counter() - t0) * 1e3:.2f} ms, mean {img.mean():.6g}", flush=True)
