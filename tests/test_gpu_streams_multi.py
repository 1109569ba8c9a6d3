"""Stream ordering of device-output renders, per-kernel resident grids, and the multi-GPU
driver (rt_multi_*) on the GPU.

* rt_render_tiles with stream NULL runs on the HIP null stream = torch's default stream, so
  work torch queues after the call (a clone, a gather) sees the finished image (camera.h:169-174:
  the image exists before anything reads it).
* two pending renders on different streams do not overwrite each other's inputs.
* every persistent kernel gets its own resident grid (occupancy query per kernel).
* rt_multi: the image tiled over devices and gathered (RCCL with distinct devices; device copies
  when a device repeats, which is how N = 2, 4, 8 ranks run on a one-GPU box) is bit-identical
  to a one-context render, and camera::render(of, world, light) through camera::devices_
  writes the same PPM.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
import rt_amd
from rt_amd import abi, plugin, scenes

pytestmark = pytest.mark.gpu
F32, F64 = abi.RT_PREC_F32, abi.RT_PREC_F64


@pytest.fixture(scope="module")
def ctx():
    c = rt_amd.Context(0)
    yield c
    c.close()


def test_device_output_is_ordered_on_torch_default_stream(ctx):
    import torch
    desc, cam, _, _ = scenes.cornell_box(width=64)
    ctx.upload(desc)
    host = ctx.render(cam, 256, 50, seed=4, precision=F32)
    out = torch.full((64 * 64, 3), -1.0, dtype=torch.float32, device="cuda:0")
    ctx.render_tiles(cam, ctx.params(256, 50, 4, F32), [(0, 0, 64, 64)], out.data_ptr(), 1,
                     torch.cuda.current_stream().cuda_stream)
    snap = out.clone()  # queued right behind the render on the same (default) stream: no sync
    assert np.array_equal(snap.cpu().numpy().reshape(host.shape), host)
    # the same on a side stream
    s = torch.cuda.Stream()
    out2 = torch.full((64 * 64, 3), -1.0, dtype=torch.float32, device="cuda:0")
    torch.cuda.current_stream().synchronize()
    with torch.cuda.stream(s):
        ctx.render_tiles(cam, ctx.params(256, 50, 4, F32), [(0, 0, 64, 64)], out2.data_ptr(), 1, s.cuda_stream)
        snap2 = out2.clone()
    s.synchronize()
    assert np.array_equal(snap2.cpu().numpy().reshape(host.shape), host)


def test_pending_render_on_another_stream_keeps_its_inputs(ctx):
    # render A (tiles A, camera A) pending on stream 1, then render B (other tiles, other camera) on
    # stream 2: B must not rewrite the pixel map / camera A's kernels are still reading
    import torch
    from rt_amd.scene import perspective
    desc, cam, _, _ = scenes.cornell_box(width=64)
    cam_b = perspective(64, 1.0, (300, 250, -780), (278, 278, 0), 1, 40.0)
    ctx.upload(desc)
    tiles_a, tiles_b = [(0, 0, 64, 32)], [(0, 32, 64, 32), (0, 0, 16, 16)]
    ref_a = ctx.render(cam, 128, 50, seed=2, precision=F32, tiles=tiles_a)
    ref_b = ctx.render(cam_b, 128, 50, seed=2, precision=F32, tiles=tiles_b)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    oa = torch.full((64 * 32, 3), -1.0, device="cuda:0")
    ob = torch.full((64 * 32 + 256, 3), -1.0, device="cuda:0")
    torch.cuda.synchronize()
    p = ctx.params(128, 50, 2, F32)
    ctx.render_tiles(cam, p, tiles_a, oa.data_ptr(), 1, s1.cuda_stream)
    ctx.render_tiles(cam_b, p, tiles_b, ob.data_ptr(), 1, s2.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(oa.cpu().numpy(), ref_a)
    assert np.array_equal(ob.cpu().numpy(), ref_b)


FRESH = """
import sys
sys.path.insert(0, {py!r})
import rt_amd
from rt_amd import scenes, abi
desc, cam, _, _ = scenes.cornell_box(width=64)
c = rt_amd.Context(0)
c.upload(desc)
c.render(cam, 4, 8, precision=abi.RT_PREC_F32)
print("LANES", c.stats().grid_lanes)
c.close()
"""


def test_resident_grid_is_per_kernel():
    # the lens camera selects the extended (CAMX) persistent kernel, whose register budget differs
    # from the plain Cornell kernel's; rendering it first must not cap the later kernel's grid
    from test_gpu_parity import _camera_variants
    py = os.path.join(abi.PKG_DIR, "python")
    r = subprocess.run([sys.executable, "-c", FRESH.format(py=py)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    fresh = int([l for l in r.stdout.split("\n") if l.startswith("LANES")][0].split()[1])
    desc, cam, _, _ = scenes.cornell_box(width=64)
    c = rt_amd.Context(0)
    c.upload(desc)
    c.render(_camera_variants()["lens"], 4, 8, precision=F32)
    lens_lanes = c.stats().grid_lanes
    c.render(cam, 4, 8, precision=F32)
    plain_lanes = c.stats().grid_lanes
    c.close()
    assert plain_lanes == fresh > 0
    assert lens_lanes > 0 and lens_lanes != plain_lanes  # different kernels, different occupancy


def test_multi_single_device_rccl_matches_context(ctx):
    m = rt_amd.Multi([0])
    assert m.uses_rccl  # one-rank RCCL communicator (ncclCommInitAll) + ncclGather
    for name, w, spp, depth in [("cornell_box", 70, 16, 8), ("cornell_box_with_volume", 64, 8, 5)]:
        desc, cam, _, _ = scenes.SCENES[name](width=w)
        m.upload(desc)
        ctx.upload(desc)
        for prec in (F32, F64):
            got = m.render(cam, spp, depth, seed=3, precision=prec)
            want = ctx.render(cam, spp, depth, seed=3, precision=prec)
            assert np.array_equal(got, want), (name, prec)
    st = m.stats(0)
    assert st.samples > 0 and st.aux_ms > 0
    m.close()


@pytest.mark.parametrize("n", [2, 4, 8])
def test_multi_ranks_are_bit_identical(ctx, n):
    # n ranks on the one device of this box (device-copy gather): same tiles, same unpack as on n GPUs
    desc, cam, _, _ = scenes.cornell_box(width=100)
    m = rt_amd.Multi([0] * n)
    assert not m.uses_rccl
    m.upload(desc)
    ctx.upload(desc)
    want = ctx.render(cam, 8, 8, seed=5, precision=F32)
    for ts in (0, 16, 64):
        assert np.array_equal(m.render(cam, 8, 8, seed=5, precision=F32, tile_size=ts), want), ts
    per_rank = [m.stats(r).samples for r in range(n)]
    assert sum(per_rank) == 3 * 100 * 100 * 8
    m.close()


def test_multi_matches_oracle_fp64():
    desc, cam, _, _ = scenes.cornell_box(width=40)
    m = rt_amd.Multi([0, 0])
    m.upload(desc)
    img = m.render(cam, 8, 8, seed=6, precision=F64)
    m.close()
    ref, _ = oracle.render(oracle.from_desc(desc), cam, 8, 8, seed=6)
    assert np.all(np.abs(img - ref) <= 1e-9 * np.maximum(1.0, np.abs(ref))), np.abs(img - ref).max()


def test_camera_render_on_devices_writes_the_same_ppm(tmp_path):
    a, b, c = (str(tmp_path / f) for f in ("one.ppm", "multi1.ppm", "multi4.ppm"))
    plugin.render_ppm("cornell_box", a, width=64, spp=8, max_depth=8, seed=6, precision=F32)
    plugin.render_ppm("cornell_box", b, width=64, spp=8, max_depth=8, seed=6, precision=F32, devices=[0])
    plugin.render_ppm("cornell_box", c, width=64, spp=8, max_depth=8, seed=6, precision=F32, devices=[0, 0, 0, 0])
    ra, rb, rc = (open(p, "rb").read() for p in (a, b, c))
    assert ra == rb == rc and ra.startswith(b"P3\n64 64\n255\n")


def test_camera_keeps_its_communicator_across_renders(tmp_path):
    # camera::render with devices_ = {0} twice on the same camera: one rt_multi, one ncclCommInitAll
    lib = abi.load()
    a, b = str(tmp_path / "once.ppm"), str(tmp_path / "twice.ppm")
    plugin.render_ppm("cornell_box", a, width=48, spp=8, max_depth=8, seed=2, precision=F32, devices=[0])
    before = lib.rt_multi_comm_inits()
    plugin.render_ppm("cornell_box", b, width=48, spp=8, max_depth=8, seed=2, precision=F32, devices=[0], repeat=2)
    assert lib.rt_multi_comm_inits() - before == 1
    assert open(a, "rb").read() == open(b, "rb").read()
    # the single-device camera keeps its context the same way (same image on the second render)
    c, d = str(tmp_path / "ctx_once.ppm"), str(tmp_path / "ctx_twice.ppm")
    plugin.render_ppm("cornell_box", c, width=48, spp=8, max_depth=8, seed=2, precision=F32)
    plugin.render_ppm("cornell_box", d, width=48, spp=8, max_depth=8, seed=2, precision=F32, repeat=3)
    assert open(c, "rb").read() == open(d, "rb").read() == open(a, "rb").read()


def test_scene_copy_of_an_empty_render_is_waited_for(ctx):
    # the scene copy queued by a render that then exits early (empty tile list) must be
    # waited for by a device-output render on another stream, which does not copy it again
    import torch
    desc, cam, _, _ = scenes.cornell_box(width=64)
    other, _, _, _ = scenes.cornell_box_with_volume(width=64)
    ctx.upload(other)
    ctx.render(cam, 4, 4, seed=1, precision=F32)  # the volume scene resident
    ctx.upload(desc)
    want = rt_amd.Context(0)
    want.upload(desc)
    ref = want.render(cam, 64, 50, seed=9, precision=F32)
    want.close()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    p = ctx.params(64, 50, 9, F32)
    dummy = torch.zeros((1, 3), device="cuda:0")
    ctx.render_tiles(cam, p, [(0, 0, 0, 0)], dummy.data_ptr(), 1, s1.cuda_stream)  # copies the scene, renders nothing
    out = torch.full((64 * 64, 3), -1.0, device="cuda:0")
    ctx.render_tiles(cam, p, [(0, 0, 64, 64)], out.data_ptr(), 1, s2.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(ref.shape), ref)


def _device_count():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_device_count() < 2, reason="needs two GPUs (runs on the first multi-GPU lease)")
def test_multi_two_devices_rccl_matches_context(ctx):
    # ncclGather across two distinct devices: rank 1's tiles land in rank 0's buffer in place
    m = rt_amd.Multi([0, 1])
    assert m.uses_rccl
    desc, cam, _, _ = scenes.cornell_box(width=100)
    m.upload(desc)
    ctx.upload(desc)
    for prec in (F32, F64):
        for ts in (0, 16, 64):
            got = m.render(cam, 8, 8, seed=5, precision=prec, tile_size=ts)
            want = ctx.render(cam, 8, 8, seed=5, precision=prec)
            assert np.array_equal(got, want), (prec, ts)
    m.close()
