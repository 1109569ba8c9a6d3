"""Multi-rank framebuffer partitioning with world_size 2 on gloo, on the CPU: the
frame driver bench.py uses (rt_amd.distributed.FrameSharding: the tile plan, the gather to rank 0
and the scatter) over a stand-in context whose render_tiles writes the oracle's pixels of the tiles
into the rank's buffer; the gathered frame equals the single-rank image exactly. The same driver on
librt_hip with both ranks on one GPU: tests/test_gpu_multiprocess.py."""
import ctypes
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


class OracleTiles:
    """render_tiles of rt_amd.Context (packed tiles into a float64 buffer) computed by the oracle."""

    def __init__(self, oracle, scene):
        self.oracle, self.scene = oracle, scene

    def render_tiles(self, cam, params, tiles, out_ptr, out_is_device, stream=None):
        img, _ = self.oracle.render(self.scene, cam, params["spp"], params["depth"], seed=params["seed"],
                                    tiles=tiles, threads=1)
        n = img.size
        ctypes.memmove(out_ptr, img.ctypes.data, n * 8)


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [os.path.join(repo, "cpu-ray-tracing-implementation_amd", "python"), os.path.join(repo, "oracle")]
    import oracle
    from rt_amd import plugin
    from rt_amd.distributed import FrameSharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cs = plugin.ConfigScene("cornell_box", 150)
    W, H = cs.cam.image_width, cs.cam.image_height
    shard = FrameSharding(W, H, world, rank, torch.device("cpu"))
    out, fb = shard.buffers(torch.float64)
    ctx = OracleTiles(oracle, oracle.from_desc(cs.desc))
    shard.frame(ctx, cs.cam, {"spp": 2, "depth": 6, "seed": 4}, out, fb, stream=0)
    if rank == 0:
        q.put(fb.numpy())
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
