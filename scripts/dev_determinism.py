#!/usr/bin/env python3
"""Development: render one config scene several times (fp32) and report whether the images are
bit-identical, and which pixels differ from the oracle.   python scripts/dev_determinism.py NAME W SPP DEPTH SEED"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))
import numpy as np  # noqa: E402

import conftest  # noqa: E402,F401
import oracle  # noqa: E402
import rt_amd  # noqa: E402
from rt_amd import abi, plugin  # noqa: E402

name, w, spp, depth, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
cs = plugin.ConfigScene(name, w)
ctx = rt_amd.Context(0)
ctx.upload(cs.desc)
imgs = [ctx.render(cs.cam, spp, depth, seed=seed, precision=abi.RT_PREC_F32) for _ in range(4)]
for i in range(1, 4):
    d = np.argwhere((imgs[i] != imgs[0]).any(-1))
    print(f"run {i} vs run 0: {len(d)} pixels differ", d[:8].tolist())
ref, _ = oracle.render(oracle.from_desc(cs.desc), cs.cam, spp, depth, seed=seed, threads=8)
for i in range(4):
    diff = np.abs(imgs[i].astype(np.float64) - ref).max(-1)
    bad = np.argwhere(diff > 1e-3)
    print(f"run {i}: {len(bad)} px > 1e-3 from the oracle", [(p.tolist(), imgs[i][tuple(p)].tolist(), ref[tuple(p)].tolist()) for p in bad[:4]])
ctx.close()
