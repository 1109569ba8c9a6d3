#!/usr/bin/env python3
"""Development (RT_ITEM_CLOCKS build): the distribution of work-item durations of one frame -- how long the
slowest items run, i.e. the tail a persistent launch waits for once its queue is dry.
    RT_HIP_LIB=<item-clocks build> python scripts/dev_item_clocks.py --config c4 --precision f64"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rt_amd  # noqa: E402
from rt_amd import abi, plugin  # noqa: E402
from bench import CONFIGS, sponza_asset  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--precision", default="f64")
ap.add_argument("--spp", type=int, default=0)
a = ap.parse_args()
scene, width, aspect, spp, depth = CONFIGS[a.config]
spp = a.spp or spp
if scene == "sponza":
    sponza_asset()
cs = plugin.ConfigScene(scene, width, aspect)
cam = cs.cam
W, H = cam.image_width, cam.image_height
ctx = rt_amd.Context(0)
ctx.upload(cs.desc)
lib = abi.load()
prec = abi.RT_PREC_F64 if a.precision == "f64" else abi.RT_PREC_F32
clk = torch.zeros(W * H * 256, dtype=torch.int32, device="cuda")
lib.rt_dev_set_item_clocks.argtypes = [ctypes.c_void_p]
assert lib.rt_dev_set_item_clocks(clk.data_ptr()) == 0
img = ctx.render(cam, spp, depth, seed=1, precision=prec)
c = clk.cpu().numpy().view(np.uint32).astype(np.float64) / 100.0  # us
n_items = int((c > 0).sum())
c = c[: ((len(c) // (W * H)) * W * H)]
nz = c[c > 0]
print(f"{a.config} {a.precision} {spp} spp: {n_items} items, mean {nz.mean():.1f} us, p50 {np.percentile(nz, 50):.1f}, "
      f"p99 {np.percentile(nz, 99):.1f}, p99.99 {np.percentile(nz, 99.99):.1f}, max {nz.max():.1f} us")
per = c.reshape(-1, W * H)
chunks = int((per.sum(1) > 0).sum())
pix = per[:chunks].sum(0)
order = np.argsort(-pix)
print("slowest pixels (local index, x, y, us over all their items, slowest item us):")
for i in order[:12]:
    print(f"  {i} ({i % W}, {i // W}) {pix[i]:.0f} {per[:chunks, i].max():.0f}")
print("top-1000 pixels' share of the item time:", f"{pix[order[:1000]].sum() / pix.sum():.4f}")
