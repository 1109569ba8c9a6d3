"""Known-answer tests of the oracle's primitives against independent numpy
restatements of the reference formulas, and the oracle's own invariances."""
import ctypes
import math

import numpy as np
import pytest

import oracle

D3 = ctypes.c_double * 3


def arr(*v):
    return D3(*[float(x) for x in v])


def test_sphere_hit_kat():  # sphere.h:40-74
    out = (ctypes.c_double * 9)()
    assert oracle.lib().orc_kat_sphere_hit(arr(0, 0, 0), 1.0, arr(0, 0, -5), arr(0, 0, 2), 0.001, math.inf, out)
    t, p, n, u, v = out[0], out[1:4], out[4:7], out[7], out[8]
    assert t == pytest.approx(2.0)  # |d| = 2: t is in units of the unnormalised direction
    assert p == pytest.approx([0, 0, -1])
    assert n == pytest.approx([0, 0, -1])
    # get_sphere_uv(outward normal (0,0,-1)): theta = acos(0), phi = atan2(1, 0) + pi
    assert u == pytest.approx((math.atan2(1, 0) + math.pi) / (2 * math.pi))
    assert v == pytest.approx(0.5)
    # inside the sphere: the far root, normal flipped towards the ray
    assert oracle.lib().orc_kat_sphere_hit(arr(0, 0, 0), 1.0, arr(0, 0, 0), arr(1, 0, 0), 0.001, math.inf, out)
    assert out[0] == pytest.approx(1.0) and list(out[4:7]) == pytest.approx([-1, 0, 0])
    # both roots outside the interval
    assert not oracle.lib().orc_kat_sphere_hit(arr(0, 0, 0), 1.0, arr(0, 0, -5), arr(0, 0, 1), 0.001, 3.0, out)


def test_quad_hit_kat():  # quad.h:30-64
    out = (ctypes.c_double * 9)()
    q, u, v = arr(0, 0, 0), arr(2, 0, 0), arr(0, 4, 0)
    assert oracle.lib().orc_kat_quad_hit(q, u, v, arr(0.5, 1, -3), arr(0, 0, 1), 0.001, math.inf, out)
    assert out[0] == pytest.approx(3.0)
    assert list(out[7:9]) == pytest.approx([0.25, 0.25])  # (alpha, beta) in the quad's u, v
    assert list(out[4:7]) == pytest.approx([0, 0, -1])  # cross(u, v) = +z, flipped to face the ray
    # closed interval: an edge hit counts, just outside does not
    assert oracle.lib().orc_kat_quad_hit(q, u, v, arr(2, 4, -1), arr(0, 0, 1), 0.001, math.inf, out)
    assert not oracle.lib().orc_kat_quad_hit(q, u, v, arr(2.0000001, 1, -1), arr(0, 0, 1), 0.001, math.inf, out)
    # parallel ray: t is +-inf or NaN and is rejected
    assert not oracle.lib().orc_kat_quad_hit(q, u, v, arr(0.5, 1, -1), arr(1, 0, 0), 0.001, math.inf, out)


def test_triangle_hit_kat():  # triangle.h:8-40
    out = (ctypes.c_double * 7)()
    p0, p1, p2 = arr(0, 0, 0), arr(1, 0, 0), arr(0, 1, 0)
    assert oracle.lib().orc_kat_triangle_hit(p0, p1, p2, arr(0.2, 0.2, 1), arr(0, 0, -2), 0.001, math.inf, out)
    assert out[0] == pytest.approx(0.5)
    assert list(out[4:7]) == pytest.approx([0, 0, 1])
    assert not oracle.lib().orc_kat_triangle_hit(p0, p1, p2, arr(0.6, 0.6, 1), arr(0, 0, -1), 0.001, math.inf, out)


def np_onb(n):  # onb.h:20-28
    y = n / np.linalg.norm(n)
    a = np.array([0, 0, 1.0]) if abs(y[0]) > 0.9 else np.array([1.0, 0, 0])
    z = np.cross(y, a)
    z /= np.linalg.norm(z)
    return np.cross(y, z), y, z


@pytest.mark.parametrize("n", [(0, 1, 0), (1, 0, 0), (0.3, -0.2, 0.9), (-0.95, 0.1, 0.1)])
def test_onb_kat(n):
    out = (ctypes.c_double * 9)()
    oracle.lib().orc_kat_onb(arr(*n), out)
    x, y, z = np_onb(np.array(n, float))
    np.testing.assert_allclose(np.array(out[:]).reshape(3, 3), np.stack([x, y, z]), atol=1e-14)


def test_refract_and_schlick_kat():  # utility.h:71-76, material.h:135-139
    v = np.array([1.0, -1.0, 0]) / math.sqrt(2)
    n = np.array([0, 1.0, 0])
    out = (ctypes.c_double * 3)()
    oracle.lib().orc_kat_refract(arr(*v), arr(*n), 1 / 1.5, out)
    cos_t = min(-v @ n, 1.0)
    perp = (1 / 1.5) * (v + cos_t * n)
    par = -math.sqrt(abs(1 - perp @ perp)) * n
    np.testing.assert_allclose(out[:], perp + par, atol=1e-15)
    for c, ri in [(1.0, 1.5), (0.3, 1 / 1.5), (0.0, 1.5)]:
        r0 = ((1 - ri) / (1 + ri)) ** 2
        assert oracle.lib().orc_kat_reflectance(c, ri) == pytest.approx(r0 + (1 - r0) * (1 - c) ** 5, rel=1e-15)


def test_oracle_is_tiling_and_thread_invariant():
    sc, cam, _, _ = oracle.builtin("cornell_box", 40)
    full, _ = oracle.render(sc, cam, 4, 8, seed=11, threads=1)
    par, _ = oracle.render(sc, cam, 4, 8, seed=11, threads=4)
    assert np.array_equal(full, par)
    tiles = [(0, 0, 40, 7), (0, 7, 13, 33), (13, 7, 27, 33)]
    packed, _ = oracle.render(sc, cam, 4, 8, seed=11, tiles=tiles)
    ref = np.concatenate([full[y:y + h, x:x + w].reshape(-1, 3) for (x, y, w, h) in tiles])
    assert np.array_equal(packed, ref)


def test_oracle_sample_ranges_compose():
    # mean over [0, 8) equals the mean of the means over [0, 4) and [4, 8)
    sc, cam, _, _ = oracle.builtin("cornell_box_with_volume", 24)
    a, _ = oracle.render(sc, cam, 8, 5, seed=3)
    b, _ = oracle.render(sc, cam, 4, 5, seed=3, first_sample=0)
    c, _ = oracle.render(sc, cam, 4, 5, seed=3, first_sample=4)
    np.testing.assert_allclose(a, (b + c) / 2, rtol=1e-12, atol=1e-12)


# ---- camera models (camera.h:52-132, 244-290): the oracle paths the device is compared with
def _cam_variants():
    from rt_amd.scene import fisheye, lens, orthonormal
    return [orthonormal(24, 1.0, 555.0, (278, 278, -800), (278, 278, 0)),
            fisheye(24, 1.0, (278, 278, -600), (278, 278, 0), 1, 110.0),
            lens(24, 1.0, (278, 278, -800), (278, 278, 0), 3.0, 1000.0, 40.0)]


@pytest.mark.parametrize("k", [0, 1, 2], ids=["orthonormal", "fisheye", "lens"])
def test_oracle_camera_models(k):
    import numpy as np
    import oracle
    from rt_amd import scenes
    desc, _, _, _ = scenes.cornell_box(width=24)
    sc = oracle.from_desc(desc)
    cam = _cam_variants()[k]
    for mode in (oracle.COUNTER, oracle.COMPAT):
        img, segs = oracle.render(sc, cam, 4, 5, seed=3, mode=mode)
        assert np.isfinite(img).all() and segs > 0
        # deterministic: the same call gives the same image
        again, _ = oracle.render(sc, cam, 4, 5, seed=3, mode=mode)
        assert np.array_equal(img, again)
    # the camera model matters: a lens/orthonormal/fisheye image differs from the perspective one
    persp, _ = oracle.render(sc, scenes.cornell_box(width=24)[1], 4, 5, seed=3)
    assert not np.allclose(img, persp)


def test_lens_camera_matches_plugin():
    from rt_amd import plugin, scenes
    cs = plugin.ConfigScene("three_material_ball_with_defocus_blur", 64)
    _, cam, _, _ = scenes.three_material_ball_with_defocus_blur(width=64)
    assert bytes(cs.cam) == bytes(cam)  # camera::initialize_lens, float aspect/angles included
