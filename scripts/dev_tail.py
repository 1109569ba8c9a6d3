#!/usr/bin/env python3
"""Development: where does a small frame (one rank of eight) lose throughput? Renders a config's
full frame at its spp and at spp/8, and rank 0's tiles of a world-8 plan at several item sizes,
printing kernel time and Msamples/s for each.

    python scripts/dev_tail.py [--config c3] [--steps 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))

import torch  # noqa: E402

import rt_amd  # noqa: E402
from rt_amd import abi, plugin  # noqa: E402
from rt_amd.tiling import plan  # noqa: E402
from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--chunks", default="0,8,4")
    args = ap.parse_args()
    scene_name, width, aspect, spp, depth = CONFIGS[args.config]
    cs = plugin.ConfigScene(scene_name, width, aspect)
    cam = cs.cam
    W, H = cam.image_width, cam.image_height
    dev = torch.device("cuda", 0)
    ctx = rt_amd.Context(0)
    ctx.upload(cs.desc)
    full = plan(W, H, 1)[0][0]
    r8 = plan(W, H, 8)[0][0]
    out = torch.zeros((W * H, 3), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run(name, tiles, npix, s, chunk):
        params = ctx.params(s, depth, 1, abi.RT_PREC_F32, samples_per_item=chunk)
        ctx.render_tiles(cam, params, tiles, out.data_ptr(), 1, stream)
        torch.cuda.synchronize(dev)
        ctx.set_timing(True)
        ctx.reset_counters()
        for _ in range(args.steps):
            ctx.render_tiles(cam, params, tiles, out.data_ptr(), 1, stream)
        st = ctx.stats()
        ctx.set_timing(False)
        k = st.step_ms / args.steps
        print(json.dumps({"case": name, "chunk": chunk, "pixels": npix, "spp": s, "kernel_ms": round(k, 3),
                          "msamples_s": round(npix * s / k / 1e3, 1), "grid_lanes": st.grid_lanes}), flush=True)

    for c in [int(x) for x in args.chunks.split(",")]:
        run("full", full, W * H, spp, c)
        run("full_spp/8", full, W * H, spp // 8, c)
        run("rank0_of_8", r8, int(plan(W, H, 8)[1][0]), spp, c)
    ctx.close()


if __name__ == "__main__":
    main()
