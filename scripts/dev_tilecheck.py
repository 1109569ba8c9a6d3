"""Dev tool: is a render bit-identical across repeats, pool sizes and tilings? (rtow, wide BVH and binary BVH)"""
import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'cpu-ray-tracing-implementation_amd/python'))
import rt_amd
from rt_amd import abi, scenes
from rt_amd.tiling import pixel_index, plan
desc, cam, _, _ = scenes.rtow(width=64, aspect=1.5)
ctx = rt_amd.Context(0)
ctx.upload(desc)
W, H = cam.image_width, cam.image_height
F32 = abi.RT_PREC_F32
for rep in range(3):
    for trav in (0, abi.RT_TRAV_ORDERED):
        base = ctx.render(cam, 8, 20, seed=9, precision=F32, traversal=trav)
        pool = ctx.render(cam, 8, 20, seed=9, precision=F32, pool_slots=777, traversal=trav)
        tiles, _, _ = plan(W, H, 3, ts=16)
        fb = np.zeros((H * W, 3), dtype=base.dtype)
        for r in range(3):
            fb[pixel_index(tiles[r], W)] = ctx.render(cam, 8, 20, seed=9, precision=F32, tiles=tiles[r], traversal=trav)
        fb = fb.reshape(base.shape)
        for name, img in (("pool", pool), ("tiles", fb)):
            d = np.abs(img - base).max(-1)
            ys, xs = np.nonzero(d)
            print(rep, trav, name, int((d > 0).sum()), float(d.max()), list(zip(xs[:6].tolist(), ys[:6].tolist())), flush=True)
