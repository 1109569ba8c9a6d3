#!/usr/bin/env python3
"""Development: device time of one config's frame at several spp (fixed cost per launch vs per sample).
    python scripts/dev_spp_time.py --config c4 --precision f64 --spp 32,64,128,256"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))
import torch  # noqa: E402

import rt_amd  # noqa: E402
from rt_amd import abi, plugin  # noqa: E402
from bench import CONFIGS, sponza_asset  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--precision", default="f64")
ap.add_argument("--spp", default="32,64,128,256")
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
scene, width, aspect, _, depth = CONFIGS[a.config]
if scene == "sponza":
    sponza_asset()
cs = plugin.ConfigScene(scene, width, aspect)
cam = cs.cam
ctx = rt_amd.Context(0)
ctx.upload(cs.desc)
prec = abi.RT_PREC_F64 if a.precision == "f64" else abi.RT_PREC_F32
dt = torch.float64 if prec == abi.RT_PREC_F64 else torch.float32
out = torch.zeros((cam.image_width * cam.image_height, 3), dtype=dt, device="cuda")
tiles = [(0, 0, cam.image_width, cam.image_height)]
for spp in [int(x) for x in a.spp.split(",")]:
    p = ctx.params(spp, depth, 1, prec)
    ctx.render_tiles(cam, p, tiles, out.data_ptr(), 1, 0)
    torch.cuda.synchronize()
    ctx.set_timing(True)
    ctx.reset_counters()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        ctx.render_tiles(cam, p, tiles, out.data_ptr(), 1, 0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.reps * 1e3
    st = ctx.stats()
    ctx.set_timing(False)
    print(f"{a.config} {a.precision} spp {spp}: {wall:.2f} ms/frame, kernel {st.step_ms / a.reps:.2f} ms, "
          f"{wall / spp:.3f} ms per spp, launches {st.iterations // a.reps}", flush=True)
