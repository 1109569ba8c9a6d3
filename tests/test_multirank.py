"""Multi-rank framebuffer partitioning with world_size 2 on
gloo: the same tile plan and gather bench.py uses, each rank rendering its
tiles with the oracle, reassembles exactly the single-rank image."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [os.path.join(repo, "cpu-ray-tracing-implementation_amd", "python"), os.path.join(repo, "oracle")]
    import oracle
    from rt_amd import plugin
    from rt_amd.tiling import pixel_index, plan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cs = plugin.ConfigScene("cornell_box", 150)
    W, H = cs.cam.image_width, cs.cam.image_height
    tiles, counts, maxpix = plan(W, H, world)
    mine, _ = oracle.render(oracle.from_desc(cs.desc), cs.cam, 2, 6, seed=4, tiles=tiles[rank], threads=1)
    buf = torch.zeros((maxpix, 3), dtype=torch.float64)
    buf[:counts[rank]] = torch.from_numpy(mine)
    parts = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    if rank == 0:
        fb = np.zeros((H * W, 3))
        for r in range(world):
            fb[pixel_index(tiles[r], W)] = parts[r][:counts[r]].numpy()
        q.put(fb)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_tiles_reassemble_the_image():
    import oracle
    from rt_amd import plugin
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    fb = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    cs = plugin.ConfigScene("cornell_box", 150)
    full, _ = oracle.render(oracle.from_desc(cs.desc), cs.cam, 2, 6, seed=4)
    assert np.array_equal(fb.reshape(full.shape), full)
