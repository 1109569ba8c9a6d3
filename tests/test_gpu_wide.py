"""The wide BVH (rt_scene.h WNode, rt_device.h trace_wide): 4-wide nodes over world-level
primitives, the fp32 traversal of BVH scenes without instances or volumes (RTOW, meshes).

It runs the same primitive tests as the binary-BVH traversal, so against that path (selected by
RT_TRAV_ORDERED) images may differ only where two primitives are hit at exactly the same t, and
against the oracle the fp32 tolerance of the other paths holds.
"""
import random

import numpy as np
import pytest

import oracle
import rt_amd
from rt_amd import abi, plugin, scenes
from rt_amd.scene import SceneBuilder, perspective

pytestmark = pytest.mark.gpu

F32 = abi.RT_PREC_F32


@pytest.fixture(scope="module")
def ctx():
    c = rt_amd.Context(0)
    yield c
    c.close()


def rmse(a, b):
    return np.sqrt(((np.asarray(a, np.float64) - b) ** 2).reshape(-1, 3).mean(0))


def mixed_scene(seed, moving=False):
    """Spheres (optionally moving), triangles and quads under one bvh_node: the generic wide kernel."""
    rnd = random.Random(seed)
    s = SceneBuilder()
    mats = [s.lambertian(s.solid((rnd.random(), rnd.random(), rnd.random()))) for _ in range(3)]
    mats.append(s.metal(s.solid((0.8, 0.8, 0.8)), 0.2))
    mats.append(s.dielectric(s.solid((1, 1, 1)), 1.5))
    objs = []
    for _ in range(40):
        c = [rnd.uniform(-8, 8), rnd.uniform(0, 5), rnd.uniform(-8, 8)]
        if moving:
            objs.append(s.moving_sphere(c, [c[0], c[1] + rnd.uniform(0, 0.5), c[2]], rnd.uniform(0.2, 0.8),
                                        rnd.choice(mats)))
        else:
            objs.append(s.sphere(c, rnd.uniform(0.2, 0.8), rnd.choice(mats)))
    for _ in range(60):
        p = [rnd.uniform(-8, 8), rnd.uniform(0, 5), rnd.uniform(-8, 8)]
        objs.append(s.triangle(p, [p[0] + rnd.uniform(-2, 2), p[1] + rnd.uniform(0, 2), p[2]],
                               [p[0], p[1] + rnd.uniform(-2, 2), p[2] + rnd.uniform(-2, 2)], rnd.choice(mats)))
    for _ in range(20):
        p = [rnd.uniform(-8, 8), rnd.uniform(0, 5), rnd.uniform(-8, 8)]
        objs.append(s.quad(p, (rnd.uniform(-2, 2), rnd.uniform(0, 1), 0.3), (0.2, rnd.uniform(0, 1), rnd.uniform(-2, 2)),
                           rnd.choice(mats)))
    objs.append(s.quad((-20, -0.01, -20), (40, 0, 0), (0, 0, 40), mats[0]))
    light = s.quad((-3, 12, -3), (6, 0, 0), (0, 0, 6), s.diffuse_light(s.solid((6, 6, 6))))
    objs.append(light)
    cam = perspective(56, 1.25, (0, 7, 22), (0, 2, 0), 1, 35.0)
    return s.desc(s.bvh(objs), light=light, background=s.solid((0.2, 0.25, 0.3))), cam


def both_traversals(ctx, desc, cam, spp, depth, seed):
    ctx.upload(desc)
    wide = ctx.render(cam, spp, depth, seed=seed, precision=F32)
    binary = ctx.render(cam, spp, depth, seed=seed, precision=F32, traversal=abi.RT_TRAV_ORDERED)
    return wide.astype(np.float64), binary.astype(np.float64)


@pytest.mark.parametrize("name,kinds", [("rtow", 1), ("rtow_motion", 9)])
def test_wide_rtow_matches_binary_bvh_and_oracle(ctx, name, kinds):
    desc, cam, _, _ = scenes.SCENES[name](width=64, aspect=1.5)
    st, info, msg = abi.scene_check(desc)
    assert st == abi.RT_OK and info.wide_nodes > 0 and info.wide_kinds == kinds, msg
    wide, binary = both_traversals(ctx, desc, cam, 8, 50, 5)
    assert np.isfinite(wide).all()
    differ = np.abs(wide - binary).max(-1) > 0
    assert differ.mean() < 2e-3, int(differ.sum())  # exact-t ties only


@pytest.mark.parametrize("moving", [False, True])
def test_wide_mixed_primitives_match_oracle(ctx, moving):
    desc, cam = mixed_scene(3, moving)
    st, info, msg = abi.scene_check(desc)
    assert st == abi.RT_OK and info.wide_kinds == (15 if moving else 7), msg
    wide, binary = both_traversals(ctx, desc, cam, 64, 10, 2)
    differ = np.abs(wide - binary).max(-1) > 0
    assert differ.mean() < 2e-3, int(differ.sum())
    if not moving:  # moving spheres keep the reference's normals from center_ = 0 (sphere.h:69): radiance
        # blows up along any path that touches one, so the fp32/fp64 comparison is ill-conditioned there
        ref, _ = oracle.render(oracle.from_desc(desc), cam, 64, 10, seed=2, threads=8)
        assert (rmse(wide, ref) < 1e-4).all(), rmse(wide, ref)


def test_wide_mesh_from_global_memory(ctx, tmp_path, monkeypatch):
    # 262,267 triangles: the tree does not fit the LDS budget, nodes and triangles come from HBM
    from rt_amd import synth_gltf
    monkeypatch.setenv("RT_SPONZA_GLTF", synth_gltf.write_sponza_standin(str(tmp_path)))
    cs = plugin.ConfigScene("sponza", 64, 16.0 / 9.0)
    st, info, msg = abi.scene_check(cs.desc)
    assert st == abi.RT_OK and info.wide_kinds == 6 and info.wide_nodes > 10000, msg  # triangles + the light quad
    # a lane may need more stack entries than the 24 kept in LDS (rtd::kWideLdsStack): the entries past
    # them go to the spill area in HBM, so this render runs that path too
    assert info.wide_stack > 24, info.wide_stack
    wide, binary = both_traversals(ctx, cs.desc, cs.cam, 4, 5, 3)
    differ = np.abs(wide - binary).max(-1) > 0
    assert differ.mean() < 5e-3, int(differ.sum())  # shared mesh edges: exact-t ties
    assert (rmse(wide, binary) < 1e-4).all(), rmse(wide, binary)


def test_wide_schedule_invariance(ctx):
    # pool size and tiling do not change the image (keys are per pixel and sample)
    desc, cam, _, _ = scenes.rtow(width=64, aspect=1.5)
    ctx.upload(desc)
    base = ctx.render(cam, 8, 20, seed=9, precision=F32)
    assert np.array_equal(ctx.render(cam, 8, 20, seed=9, precision=F32, pool_slots=777), base)
    from rt_amd.tiling import pixel_index, plan
    W, H = cam.image_width, cam.image_height
    tiles, _, _ = plan(W, H, 3, ts=16)
    fb = np.zeros((H * W, 3), dtype=base.dtype)
    for r in range(3):
        fb[pixel_index(tiles[r], W)] = ctx.render(cam, 8, 20, seed=9, precision=F32, tiles=tiles[r])
    d = np.abs(fb.reshape(base.shape) - base).max(-1)
    assert not d.any(), (int((d > 0).sum()), float(d.max()), np.argwhere(d)[:8].tolist())


def test_pixel_map_follows_the_last_tiles_height(ctx):
    # two tile lists equal but for the last tile's height (images of one width): the cached pixel
    # map must not be reused (round-2 fix; the tile entry {x0, y0, width, first} has no height)
    desc, cam, _, _ = scenes.rtow(width=64, aspect=1.5)
    ctx.upload(desc)
    W, H = cam.image_width, cam.image_height
    fresh = ctx.render(cam, 2, 5, seed=4, precision=F32)
    # left half then right half: every map entry now in column-half order
    ctx.render(cam, 2, 5, seed=4, precision=F32, tiles=[(0, 0, W // 2, H), (W // 2, 0, W - W // 2, H)])
    ctx.render(cam, 2, 5, seed=4, precision=F32, tiles=[(0, 0, W, H // 2)])  # rewrites the first half only
    again = ctx.render(cam, 2, 5, seed=4, precision=F32, tiles=[(0, 0, W, H)])  # same entry as the last list
    assert np.array_equal(again.reshape(fresh.shape), fresh)


def both_traversals_f64(ctx, desc, cam, spp, depth, seed):
    ctx.upload(desc)
    wide = ctx.render(cam, spp, depth, seed=seed, precision=abi.RT_PREC_F64)
    binary = ctx.render(cam, spp, depth, seed=seed, precision=abi.RT_PREC_F64, traversal=abi.RT_TRAV_ORDERED)
    return wide, binary


@pytest.mark.parametrize("which", ["rtow", "mixed", "sponza"])
def test_wide_fp64_matches_binary_and_oracle(ctx, which, tmp_path, monkeypatch):
    # fp64 rays over the float boxes (round 3): the slabs are widened for the rounding of the ray to float,
    # so they only cull; the primitive tests are the fp64 ones, and the closest hits equal the fp64 binary
    # BVH's (ties aside) -- the LDS-resident sphere tree (rtow), the all-kinds kernel (mixed) and the tree
    # in HBM with its spill area (the Sponza stand-in)
    if which == "rtow":
        desc, cam, _, _ = scenes.rtow(width=64, aspect=1.5)
        spp, depth, seed = 8, 50, 5
    elif which == "mixed":
        desc, cam = mixed_scene(3, False)
        spp, depth, seed = 16, 10, 2
    else:
        from rt_amd import synth_gltf
        monkeypatch.setenv("RT_SPONZA_GLTF", synth_gltf.write_sponza_standin(str(tmp_path)))
        cs = plugin.ConfigScene("sponza", 64, 16.0 / 9.0)
        desc, cam, spp, depth, seed = cs.desc, cs.cam, 4, 5, 3
    wide, binary = both_traversals_f64(ctx, desc, cam, spp, depth, seed)
    assert np.isfinite(wide).all()
    differ = np.abs(wide - binary).max(-1) > 1e-9 * np.maximum(1.0, np.abs(binary).max(-1))
    assert differ.mean() < 5e-3, int(differ.sum())
    if which != "sponza":  # (the oracle's x-median tree over 262k triangles takes minutes)
        ref, _ = oracle.render(oracle.from_desc(desc), cam, spp, depth, seed=seed, threads=8)
        bad = (np.abs(wide - ref) > 1e-9 * np.maximum(1.0, np.abs(ref))).any(-1)
        assert bad.mean() < 5e-3, (int(bad.sum()), float(np.abs(wide - ref).max()))
