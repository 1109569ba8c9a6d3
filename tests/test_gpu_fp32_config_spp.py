"""fp32 parity at the north-star tolerance (per-channel RMSE < 1e-4 against the fp64 oracle) for
the scenes whose low-spp checks in test_gpu_parity.py compare only statistics or looser bounds:
gloss, the procedural and picture textures, the lens camera, the glTF meshes.

fp32 follows the oracle's fp64 paths sample for sample except where rounding sends a ray across
an edge (a triangle edge of a mesh, a checker line, a glass/metal chain that bends the other way).
Such a sample moves its pixel by ~value/spp, so the RMSE of the few divergent pixels shrinks with
spp: these tests run at sample counts near the reference's own configs (main.cc) on small images,
where the oracle finishes in seconds. The low-spp tests stay as they are: they check the same
scenes' fp64 path to 1e-9.
"""
import os

import numpy as np
import pytest

import oracle
import rt_amd
from rt_amd import abi, plugin, scenes

pytestmark = pytest.mark.gpu

F32 = abi.RT_PREC_F32
GOLDEN_ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "assets")
TOL = 1e-4  # north_star: per-channel RMSE against the fp64 reference


@pytest.fixture(scope="module")
def ctx():
    c = rt_amd.Context(0)
    yield c
    c.close()


def fp32_vs_oracle(ctx, desc, cam, spp, depth, seed):
    ctx.upload(desc)
    img = ctx.render(cam, spp, depth, seed=seed, precision=F32).astype(np.float64)
    ref, _ = oracle.render(oracle.from_desc(desc), cam, spp, depth, seed=seed, threads=8)
    err = np.sqrt(((img - ref) ** 2).reshape(-1, 3).mean(0))
    div = int((np.abs(img - ref).max(-1) > 1e-3).sum())
    return err, div, img, ref


def check(name, err, div, npix):
    print(f"{name}: fp32 rmse {err} divergent px {div}/{npix}")
    assert np.isfinite(err).all() and (err < TOL).all(), (name, err, div)


def test_gloss_fp32_at_config_spp(ctx):
    # material.h:145-185 (gloss) in the Cornell box at 256 spp
    desc, cam, _, _ = scenes.cornell_glossy(width=40)
    err, div, img, _ = fp32_vs_oracle(ctx, desc, cam, 256, 8, 6)
    check("gloss", err, div, img.shape[0] * img.shape[1])


@pytest.mark.parametrize("name", ["test_perlin_noise", "test_value_noise", "test_worley_noise", "test_voronoi_noise",
                                  "perlin_texture_ball"])
def test_noise_textures_fp32_at_config_spp(ctx, name):
    # texture.h:80-119 / noise.h: fp32 hit points feed the fp64 noise evaluation
    cs = plugin.ConfigScene(name, 40)
    # perlin_texture_ball (main.cc:402-437) also has a glass sphere and 400 boxes (heights from rand()
    # after srand(1), as in the reference's process): a sample crossing a box edge the other way moves
    # its pixel by ~2/spp, so it runs at 1024 spp
    spp = 1024 if name == "perlin_texture_ball" else 256
    err, div, img, _ = fp32_vs_oracle(ctx, cs.desc, cs.cam, spp, 8, 8)
    check(name, err, div, img.shape[0] * img.shape[1])


def test_defocus_blur_fp32_at_config_spp(ctx):
    # main.cc:87-103 (lens camera, camera.h:102-132, 276-290) at 256 spp
    cs = plugin.ConfigScene("three_material_ball_with_defocus_blur", 48)
    err, div, img, _ = fp32_vs_oracle(ctx, cs.desc, cs.cam, 256, 10, 2)
    check("defocus", err, div, img.shape[0] * img.shape[1])


def test_skybox_fisheye_fp32_at_config_spp(ctx, tmp_path, monkeypatch):
    # main.cc:173-183: the fisheye camera (camera.h:259-275) looking at a glass sphere (refraction index 1)
    # under a picture-texture skybox (camera.h:180-190) at 256 spp; the skybox is written as a PFM here
    # (the reference's bathroom.exr is not in its checkout)
    from test_plugin import _write_assets
    _write_assets(tmp_path)
    monkeypatch.setenv("RT_ASSETS", str(tmp_path))
    cs = plugin.ConfigScene("skybox_and_fisheye", 40)
    err, div, img, _ = fp32_vs_oracle(ctx, cs.desc, cs.cam, 256, 5, 3)
    check("skybox_fisheye", err, div, img.shape[0] * img.shape[1])


def test_earthmap_fp32_at_config_spp(ctx, monkeypatch):
    # main.cc:185-196: the reference's earthmap.jpg on the moving sphere, magenta skybox
    monkeypatch.setenv("RT_ASSETS", GOLDEN_ASSETS)
    cs = plugin.ConfigScene("skybox_and_motion_blur", 48)
    err, div, img, _ = fp32_vs_oracle(ctx, cs.desc, cs.cam, 256, 5, 3)
    check("earthmap", err, div, img.shape[0] * img.shape[1])


def test_glass_fox_fp32_at_config_spp(ctx, monkeypatch):
    # main.cc:345-400 on the reference's Fox asset (576 glass triangles) at 256 spp
    monkeypatch.setenv("RT_ASSETS", GOLDEN_ASSETS)
    cs = plugin.ConfigScene("glass_fox", 48)
    err, div, img, _ = fp32_vs_oracle(ctx, cs.desc, cs.cam, 256, 5, 3)
    check("glass_fox", err, div, img.shape[0] * img.shape[1])


def test_sponza_standin_fp32_at_config_spp(ctx, tmp_path, monkeypatch):
    # C4 (main.cc:439-498) at its own 256 spp and depth 5 on a 48x27 crop of the frame
    from rt_amd import synth_gltf
    monkeypatch.setenv("RT_SPONZA_GLTF", synth_gltf.write_sponza_standin(str(tmp_path)))
    cs = plugin.ConfigScene("sponza", 48, 16.0 / 9.0)
    err, div, img, _ = fp32_vs_oracle(ctx, cs.desc, cs.cam, 256, 5, 3)
    check("sponza", err, div, img.shape[0] * img.shape[1])


def fox_triangles():
    """The reference's Fox.gltf POSITION accessor (576 non-indexed float triangles) read directly,
    as rt/gltf_loader.h and the reference's loader do (gltf_loader.h:256-810)."""
    import json
    d = os.path.join(GOLDEN_ASSETS, "Fox", "glTF")
    g = json.load(open(os.path.join(d, "Fox.gltf")))
    acc = g["accessors"][g["meshes"][-1]["primitives"][0]["attributes"]["POSITION"]]
    bv = g["bufferViews"][acc["bufferView"]]
    raw = open(os.path.join(d, g["buffers"][0]["uri"]), "rb").read()
    off = bv.get("byteOffset", 0) + acc.get("byteOffset", 0)
    pts = np.frombuffer(raw, dtype="<f4", count=acc["count"] * 3, offset=off).reshape(-1, 3).astype(np.float64)
    return pts.reshape(-1, 3, 3)


def test_fox_mesh_lit_fp32_and_fp64(ctx):
    # The glass_fox scene sees only the uniform (magenta) sky through its glass, so any path through
    # the glass gives the same colour and its image does not test the mesh hits. Here the same 576
    # triangles are diffuse and metal under a quad light over a checker floor, seen from closer than
    # main.cc:395's camera so the mesh covers ~20 % of the frame: every triangle hit changes the pixel.
    from rt_amd.scene import SceneBuilder, perspective
    tris = fox_triangles()
    assert tris.shape == (576, 3, 3)
    s = SceneBuilder()
    fur = s.lambertian(s.solid((0.8, 0.45, 0.2)))
    chrome = s.metal(s.solid((0.9, 0.9, 0.9)), 0.05)
    objs = [s.triangle(t[0], t[1], t[2], chrome if i % 7 == 0 else fur) for i, t in enumerate(tris)]
    objs.append(s.quad((-300, -0.2, -300), (600, 0, 0), (0, 0, 600),
                       s.lambertian(s.checker((0.2, 0.3, 0.1), (0.9, 0.9, 0.9), 8.0))))
    light = s.quad((-80, 260, -80), (160, 0, 0), (0, 0, 160), s.diffuse_light(s.solid((12, 12, 12))))
    objs.append(light)
    desc = s.desc(s.bvh(objs), light=light, background=s.solid((0.15, 0.2, 0.3)))
    cam = perspective(48, 1.0, (140, 60, 100), (0, 35, -10), 1, 45.0)
    ctx.upload(desc)
    img64 = ctx.render(cam, 16, 5, seed=5, precision=abi.RT_PREC_F64)
    ref16, _ = oracle.render(oracle.from_desc(desc), cam, 16, 5, seed=5, threads=8)
    bad = np.abs(img64 - ref16) > 1e-9 * np.maximum(1.0, np.abs(ref16))
    # our SAH tree vs the reference's x-median tree: only exact-t ties (shared mesh edges) may differ
    assert bad.any(-1).mean() < 0.01, np.abs(img64 - ref16).max()
    # a sample whose fp32 ray crosses a mesh edge the other way moves its pixel by ~value/spp: at 256
    # spp one such pixel of 2,304 left the RMSE at 9.8e-5, so this runs at 1024
    err, div, img, ref = fp32_vs_oracle(ctx, desc, cam, 1024, 5, 5)
    # most of the frame is lit geometry (mesh and floor), not background
    assert np.mean(np.abs(ref - np.array([0.15, 0.2, 0.3])).max(-1) > 1e-3) > 0.3
    check("fox_lit", err, div, img.shape[0] * img.shape[1])


def terrain_triangles(n=64, size=400.0, amp=30.0, seed=4):
    """A seeded height field of 2 n^2 triangles (8,192 at n = 64)."""
    rng = np.random.default_rng(seed)
    x = np.linspace(-size / 2, size / 2, n + 1)
    X, Z = np.meshgrid(x, x, indexing="ij")
    H = amp * (np.sin(X / 37.0) * np.cos(Z / 23.0) + 0.3 * rng.standard_normal(X.shape))
    P = np.stack([X, H, Z], -1)
    a, b, c, d = P[:-1, :-1], P[1:, :-1], P[1:, 1:], P[:-1, 1:]
    first = np.stack([a, b, c], -2).reshape(-1, 3, 3)
    second = np.stack([a, c, d], -2).reshape(-1, 3, 3)
    return np.stack([first, second], 1).reshape(-1, 3, 3)


def test_mesh_tree_in_hbm_lit_fp64_and_fp32(ctx):
    # C4's kernel (main.cc:439-498: triangles under a quad light, the wide tree in HBM) on a lit scene:
    # the C4 stand-in frame is dim (its light sits above the grids that close the atrium), so its own
    # parity rows compare mostly black pixels. 8,192 triangles are 24,576 primitive words, past the
    # 4,096 an LDS-resident tree may hold (rt_kernels.hip launch_wide_k), so this takes the HBM tree --
    # the C4 stand-in's kernel (triangles + quad) -- and every pixel sees lit triangles.
    from rt_amd.scene import SceneBuilder, perspective
    tris = terrain_triangles()
    assert tris.shape == (8192, 3, 3)
    s = SceneBuilder()
    ground = s.lambertian(s.solid((0.7, 0.6, 0.5)))
    chrome = s.metal(s.solid((0.9, 0.9, 0.9)), 0.1)
    objs = [s.triangle(t[0], t[1], t[2], chrome if i % 11 == 0 else ground) for i, t in enumerate(tris)]
    light = s.quad((-60, 150, -60), (120, 0, 0), (0, 0, 120), s.diffuse_light(s.solid((15, 15, 15))))
    objs.append(light)
    desc = s.desc(s.bvh(objs), light=light, background=s.solid((0.05, 0.07, 0.1)))
    cam = perspective(32, 1.0, (180, 140, 160), (0, 0, 0), 1, 50.0)
    ctx.upload(desc)
    img64 = ctx.render(cam, 32, 5, seed=3, precision=abi.RT_PREC_F64)
    ref32, _ = oracle.render(oracle.from_desc(desc), cam, 32, 5, seed=3, threads=8)
    assert ref32.mean() > 0.2 and (ref32.max(-1) > 1e-3).mean() > 0.95  # lit, not background
    bad = np.abs(img64 - ref32) > 1e-9 * np.maximum(1.0, np.abs(ref32))
    # our SAH tree vs the reference's x-median tree: only exact-t ties (shared grid edges) may differ
    assert bad.any(-1).mean() < 0.01, np.abs(img64 - ref32).max()
    err, div, img, ref = fp32_vs_oracle(ctx, desc, cam, 1024, 5, 3)
    check("terrain_hbm", err, div, img.shape[0] * img.shape[1])


def test_c4_lit_standin_tiles_match_oracle(ctx, tmp_path, monkeypatch):
    # C4's tree and kernel on lit pixels: `sponza_lit` is the C4 stand-in (main.cc:439-498: 262,267 triangles
    # in HBM, the reference's light at y = 1200) plus an unsampled light under the stand-in's grid over the
    # camera (scenes/config_scenes.cpp), whose own frame is nearly black. Four 16x16 tiles of the full
    # 1920x1080 frame at depth 5: fp64 within 1e-9 of the oracle, fp32 RMSE < 1e-4 (at 1024 spp, where a
    # sample that crosses a triangle edge the other way moves its pixel by ~value/1024).
    from rt_amd import synth_gltf
    monkeypatch.setenv("RT_SPONZA_GLTF", synth_gltf.write_sponza_standin(str(tmp_path)))
    cs = plugin.ConfigScene("sponza_lit", 1920, 16.0 / 9.0)
    cam = cs.cam
    assert (cam.image_width, cam.image_height) == (1920, 1080)
    tiles = [(960, 528, 16, 16), (400, 700, 16, 16), (1504, 600, 16, 16), (64, 1040, 16, 16)]
    st, info, _ = abi.scene_check(cs.desc)
    assert st == 0 and info.triangles == 262_267 and info.wide_nodes * 48 > 40 << 10  # the HBM tree
    ref, _ = oracle.render(oracle.from_desc(cs.desc), cam, 1024, 5, seed=2, threads=16, tiles=tiles)
    assert ref.mean() > 0.05 and (ref.max(-1) > 1e-3).mean() > 0.5, ref.mean()  # lit pixels
    ctx.upload(cs.desc)
    img64 = ctx.render(cam, 1024, 5, seed=2, precision=abi.RT_PREC_F64, tiles=tiles)
    bad = (np.abs(img64 - ref) > 1e-9 * np.maximum(1.0, np.abs(ref))).any(-1)
    # our SAH tree vs the reference's x-median tree: only exact-t ties (the stand-in's coplanar duplicates)
    assert bad.mean() < 0.01, (int(bad.sum()), np.abs(img64 - ref).max())
    img32 = ctx.render(cam, 1024, 5, seed=2, precision=F32, tiles=tiles).astype(np.float64)
    err = np.sqrt(((img32 - ref) ** 2).reshape(-1, 3).mean(0))
    check("c4_lit", err, int((np.abs(img32 - ref).max(-1) > 1e-3).sum()), len(ref))
