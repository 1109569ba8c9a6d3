"""The multi-process product path (the reference's camera.h:154-172 row loop) on the
hardware a lease provides: two processes, each rendering its 16x16 tiles through librt_hip on cuda:0,
rank 0 gathering over gloo with the same driver bench.py uses (rt_amd.distributed.FrameSharding).
The gathered frame must be bit-identical to a one-process render, in fp32 and fp64. The ranks come
from the forkserver conftest.py starts before this process touches the GPU."""
import multiprocessing as mp
import socket

import numpy as np
import pytest

import rt_amd
from rt_amd import abi, plugin

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("scene,width,spp,depth", [("cornell_box", 800, 32, 50), ("rtow", 240, 16, 50)],
                         ids=["c2_geometry", "rtow"])
def test_two_processes_gather_the_one_process_frame(scene, width, spp, depth):
    import os

    import mp_gpu_worker
    if os.environ.get("RT_FORKSERVER_EARLY") != "1":  # never let multiprocessing start the server after HIP is initialised
        pytest.skip("the forkserver was not started by conftest.pytest_configure")
    mctx = mp.get_context("forkserver")
    q = mctx.Queue()
    port = _free_port()
    world, seed = 2, 9
    procs = [mctx.Process(target=mp_gpu_worker.render_rank, args=(r, world, port, q, scene, width, spp, depth, seed))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        status, frames, counts = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    assert status == "ok", frames
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert min(counts) > 0
    cs = plugin.ConfigScene(scene, width)
    ctx = rt_amd.Context(0)
    ctx.upload(cs.desc)
    for prec in (abi.RT_PREC_F32, abi.RT_PREC_F64):
        one = ctx.render(cs.cam, spp, depth, seed=seed, precision=prec)
        got = frames[prec].reshape(one.shape)
        assert got.dtype == one.dtype
        assert np.array_equal(got, one), (prec, int((got != one).any(-1).sum()))
    ctx.close()
