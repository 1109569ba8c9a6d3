"""The fp32 flat program (rt_scene.h FlatQuad/FlatBox, rt_device.h trace_flat).

Scenes whose linear program holds only axis-aligned quads (world level or under
translate-only instances) are traced in fp32 as world-space quads grouped by plane axis,
with every lambertian `box()` (quad.h:91-112) as one slab test. The flat program is not
the reference's list order, so it can differ from the ordered (reference-order) traversal
only in exact-t ties and rounding: both are compared with the fp64 oracle at the
north-star tolerance, and with each other.
"""
import numpy as np
import pytest

import oracle
import rt_amd
from rt_amd import abi, scenes
from rt_amd.scene import SceneBuilder, perspective

pytestmark = pytest.mark.gpu

F32 = abi.RT_PREC_F32


@pytest.fixture(scope="module")
def ctx():
    c = rt_amd.Context(0)
    yield c
    c.close()


def rmse(a, b):
    return np.sqrt(((a - b) ** 2).reshape(-1, 3).mean(0))


def cornell_walls(s):
    red = s.lambertian(s.solid((.65, .05, .05)))
    white = s.lambertian(s.solid((0.73, 0.73, 0.73)))
    green = s.lambertian(s.solid((.12, .45, .15)))
    light = s.diffuse_light(s.solid((15, 15, 15)))
    w = [s.quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green), s.quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red),
         s.quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white),
         s.quad((555, 555, 555), (-555, 0, 0), (0, 0, -555), white),
         s.quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white)]
    lq = s.quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), light)
    return w, lq, white


def metal_box_scene(width):
    """Cornell walls + a translated metal box (not lambertian: its quads stay separate flat
    quads) + a translated lambertian box with a checker texture (a slab record)."""
    s = SceneBuilder()
    w, lq, white = cornell_walls(s)
    metal = s.metal(s.solid((0.8, 0.85, 0.88)), 0.0)
    chk = s.lambertian(s.checker((0.2, 0.3, 0.1), (0.9, 0.9, 0.9), 20.0))
    w.append(s.translate(s.box((0, 0, 0), (165, 330, 165), metal), (265, 0, 295)))
    w.append(s.translate(s.translate(s.box((0, 0, 0), (165, 165, 165), chk), (30, 0, 40)), (100, 0, 25)))
    w.append(lq)
    cam = perspective(width, 1.0, (278, 278, -800), (278, 278, 0), 1, 40.0)
    return s.desc(s.hlist(w), light=lq), cam


def inside_box_scene(width):
    """The camera inside a lambertian box (a slab record hit from inside: its exit faces),
    lit by a quad light inside it."""
    s = SceneBuilder()
    white = s.lambertian(s.solid((0.73, 0.6, 0.5)))
    light = s.diffuse_light(s.solid((12, 12, 12)))
    lq = s.quad((-1, 2.9, -1), (2, 0, 0), (0, 0, 2), light)
    room = s.translate(s.box((-3, -3, -3), (3, 3, 3), white), (0.25, 0, 0.5))
    cam = perspective(width, 1.0, (0, 0, -2), (0, 0.5, 0), 1, 70.0)
    return s.desc(s.hlist([room, lq]), light=lq), cam


def render_pair(ctx, desc, cam, spp, depth, seed):
    ctx.upload(desc)
    flat = ctx.render(cam, spp, depth, seed=seed, precision=F32).astype(np.float64)
    ordered = ctx.render(cam, spp, depth, seed=seed, precision=F32, traversal=abi.RT_TRAV_ORDERED).astype(np.float64)
    ref, _ = oracle.render(oracle.from_desc(desc), cam, spp, depth, seed=seed)
    return flat, ordered, ref


@pytest.mark.parametrize("name", ["cornell_box", "metal_box", "inside_box"])
def test_flat_program_matches_oracle(ctx, name):
    if name == "cornell_box":
        desc, cam, _, _ = scenes.cornell_box(width=64)
    elif name == "metal_box":
        desc, cam = metal_box_scene(64)
    else:
        desc, cam = inside_box_scene(64)
    flat, ordered, ref = render_pair(ctx, desc, cam, 16, 8, 11)
    assert (rmse(flat, ref) < 1e-4).all(), rmse(flat, ref)
    assert (rmse(ordered, ref) < 1e-4).all(), rmse(ordered, ref)
    assert (rmse(flat, ordered) < 1e-4).all(), rmse(flat, ordered)
    assert flat.max() > 0  # the scene is lit


def test_flat_program_divergence_is_rare(ctx):
    # at a realistic size, fp32 flat and fp32 ordered follow the same paths except for a
    # handful of samples that rounding moves across an edge
    desc, cam, _, _ = scenes.cornell_box(width=200)
    flat, ordered, ref = render_pair(ctx, desc, cam, 16, 10, 7)
    d = np.abs(flat - ref).max(-1)
    assert np.mean(d > 1e-3) < 5e-5, (int((d > 1e-3).sum()), d.size)
    assert (rmse(flat, ref) < 2e-4).all(), rmse(flat, ref)


def test_flat_program_invariant_to_schedule(ctx):
    desc, cam, _, _ = scenes.cornell_box(width=70)
    ctx.upload(desc)
    base = ctx.render(cam, 12, 6, seed=3, precision=F32)
    for kw in [dict(pool_slots=1000, segments_per_launch=1), dict(pool_slots=1 << 16, segments_per_launch=64),
               dict(pool_slots=333)]:
        assert np.array_equal(ctx.render(cam, 12, 6, seed=3, precision=F32, **kw), base), kw
