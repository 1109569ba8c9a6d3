#!/usr/bin/env python3
"""Predict bench.py's strong scaling on one GPU: render each rank's tiles of a world-N plan
alone (what that rank's GPU does between the barriers, minus the gather) and report the
max over ranks per N.

    python scripts/dev_scaling.py [--config c2] [--worlds 1,2,4,8] [--steps 3]
"""
import argparse
import gc
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))

import torch  # noqa: E402

import rt_amd  # noqa: E402
from rt_amd import abi, plugin  # noqa: E402
from rt_amd.tiling import TILE, plan  # noqa: E402
from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pool", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--ts", type=int, default=TILE, help="tile edge (default rt_amd.tiling.TILE)")
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    args = ap.parse_args()
    scene_name, width, aspect, spp, depth = CONFIGS[args.config]
    cs = plugin.ConfigScene(scene_name, width, aspect)
    cam = cs.cam
    W, H = cam.image_width, cam.image_height
    dev = torch.device("cuda", 0)
    ctx = rt_amd.Context(0)
    ctx.upload(cs.desc)
    prec = abi.RT_PREC_F64 if args.precision == "f64" else abi.RT_PREC_F32
    params = ctx.params(spp, depth, 1, prec, samples_per_item=args.chunk, pool_slots=args.pool)
    base = None
    for world in [int(x) for x in args.worlds.split(",")]:
        all_tiles, counts, maxpix = plan(W, H, world, ts=args.ts)
        out = torch.zeros((maxpix, 3), dtype=torch.float64 if args.precision == "f64" else torch.float32, device=dev)
        per_rank, kern = [], []
        for r in range(world):
            stream = torch.cuda.current_stream(dev).cuda_stream
            tl = abi.TileList(all_tiles[r])  # built once, as FrameSharding does (bench.py)
            ctx.render_tiles(cam, params, tl, out.data_ptr(), 1, stream)  # warmup
            torch.cuda.synchronize(dev)
            ctx.set_timing(True)
            ctx.reset_counters()
            t0 = time.perf_counter()
            gc.disable()  # (round 6: one rank's host time in a C3 8-rank run was 2-3x its kernel time)
            for _ in range(args.steps):
                ctx.render_tiles(cam, params, tl, out.data_ptr(), 1, stream)
            torch.cuda.synchronize(dev)
            per_rank.append((time.perf_counter() - t0) / args.steps * 1e3)
            gc.enable()
            kern.append(ctx.stats().step_ms / args.steps)  # the persistent kernel alone (HIP events)
            ctx.set_timing(False)
        worst = max(per_rank)
        if base is None:
            base = worst * world
        rec = {"world": world, "ms_max": round(worst, 3), "ms_mean": round(sum(per_rank) / world, 3),
               "ms_min": round(min(per_rank), 3), "kernel_ms_max": round(max(kern), 3), "pixels_max": max(counts), "pixels_min": min(counts),
               "msamples_s": round(W * H * spp / worst / 1e3, 1), "efficiency_vs_1": round(base / world / worst, 3)}
        print(json.dumps(rec), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
