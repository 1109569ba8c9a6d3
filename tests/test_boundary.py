"""The C ABI (include/rt_hip.h) without a GPU: every declared symbol is exported,
the ctypes structs match the C compiler's layout, scene compilation and its
errors, and clean failure when no device is present."""
import ctypes
import os
import re
import subprocess

import pytest

from rt_amd import abi, scenes
from rt_amd.scene import SceneBuilder

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "rt_hip.h")
STRUCTS = ["rt_object", "rt_material", "rt_texture", "rt_scene_desc", "rt_camera_desc", "rt_render_params",
           "rt_tile", "rt_counters", "rt_scene_info"]


def declared_functions():
    text = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:rt_status|void|const char\*|int32_t|uint32_t|uint64_t)\s+(rt_\w+)\(", text, re.M)))


def test_every_declared_symbol_is_exported():
    lib = abi.load()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(abi.SIGNATURES), set(names) ^ set(abi.SIGNATURES)
    assert lib.rt_abi_version() == abi.ABI_VERSION == 8


def test_struct_layout_matches_c(tmp_path):
    prog = tmp_path / "layout.c"
    prog.write_text('#include "%s"\n#include <stdio.h>\nint main(void){\n' % HDR +
                    "".join(f'printf("{s} %zu\\n", sizeof({s}));\n' for s in STRUCTS) + "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-o", str(exe), str(prog)], check=True)
    sizes = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split("\n")
                 if line)
    for s in STRUCTS:
        assert ctypes.sizeof(getattr(abi, s)) == int(sizes[s]), s


def test_context_create_without_device_fails_cleanly():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    lib = abi.load()
    h = ctypes.c_void_p()
    assert lib.rt_context_create(0, ctypes.byref(h)) == abi.RT_ERR_NO_DEVICE
    assert not h.value
    assert b"device" in lib.rt_last_error(None)


@pytest.mark.parametrize("name,quads,spheres,linear,flat", [("cornell_box", 18, 0, True, (6, 2)),
                                                            ("cornell_box_with_volume", 18, 0, True, (0, 0)),
                                                            ("three_material_ball", 0, 4, True, (0, 0)),
                                                            ("rtow", 0, 339, False, (0, 0))])
def test_scene_check_config_scenes(name, quads, spheres, linear, flat):
    desc, _, _, _ = scenes.SCENES[name](width=16)
    st, info, msg = abi.scene_check(desc)
    assert st == abi.RT_OK, msg
    assert (info.quads, info.spheres) == (quads, spheres)
    assert (info.linear_ops > 0) == linear
    # fp32 flat program: Cornell's 5 walls + light as world-space quads, its 2 translated boxes as slabs
    assert (info.flat_quads, info.flat_boxes) == flat
    if not linear:
        assert info.bvh_nodes > 0 and 1 <= info.stack_need <= 32
    # the fp32 wide BVH: only RTOW (a bvh_node of world-level spheres) gets one
    if name == "rtow":
        assert info.wide_kinds == 1 and 0 < info.wide_nodes < 339 and 1 <= info.wide_stack <= 32
        assert info.wide_prim_words == 2 * 339 + 2  # [c1, entry] [dc, r] per sphere, then two padding words
        assert info.wide_big == 1  # the r = 1000 ground, tested before the tree
    else:
        assert info.wide_nodes == 0 and info.wide_kinds == 0


def test_scene_check_wide_bvh_needs_world_level_primitives():
    # a translate/rotate instance under the BVH keeps the binary-BVH traversal (instances carry state)
    s = SceneBuilder()
    m = s.lambertian(s.solid((0.5, 0.5, 0.5)))
    objs = [s.sphere((i, 0, 0), 0.3, m) for i in range(20)]
    st, info, _ = abi.scene_check(s.desc(s.bvh(objs)))
    assert st == abi.RT_OK and info.wide_kinds == 1 and info.wide_nodes > 0
    objs.append(s.translate(s.sphere((0, 0, 0), 0.3, m), (0, 2, 0)))
    st, info, _ = abi.scene_check(s.desc(s.bvh(objs)))
    assert st == abi.RT_OK and info.wide_nodes == 0 and info.bvh_nodes > 0


def test_scene_check_volume_list_keeps_reference_order():
    desc, _, _, _ = scenes.cornell_box_with_volume(width=16)
    st, info, _ = abi.scene_check(desc)
    assert st == abi.RT_OK and info.volumes == 2 and info.instances == 2 and info.bvh_nodes == 0


def test_unsupported_material_is_rejected():
    s = SceneBuilder()
    m = s._mat(9, s.solid((1, 1, 1)))  # not a material.h kind
    st, _, msg = abi.scene_check(s.desc(s.sphere((0, 0, 0), 1, m)))
    assert st == abi.RT_ERR_UNSUPPORTED and "material kind" in msg
    # gloss (material.h:145-185) compiles for the device
    s2 = SceneBuilder()
    g = s2.gloss(s2.solid((1, 1, 1)), 0.5, 0.3)
    st, _, msg = abi.scene_check(s2.desc(s2.sphere((0, 0, 0), 1, g)))
    assert st == abi.RT_OK, msg


def test_bad_descriptors_are_rejected():
    s = SceneBuilder()
    m = s.lambertian(s.solid((1, 1, 1)))
    q = s.quad((0, 0, 0), (1, 0, 0), (0, 1, 0), m)
    st, _, msg = abi.scene_check(s.desc(q + 5))
    assert st == abi.RT_ERR_INVALID_ARGUMENT
    # a primitive without a material
    s2 = SceneBuilder()
    st, _, msg = abi.scene_check(s2.desc(s2.sphere((0, 0, 0), 1, -1)))
    assert st == abi.RT_ERR_UNSUPPORTED and "material" in msg
    # a cycle in the object graph
    s3 = SceneBuilder()
    t = s3.translate(0, (1, 0, 0))  # child 0 = itself
    st, _, msg = abi.scene_check(s3.desc(t))
    assert st != abi.RT_OK
    # a volume whose boundary mixes two different wrapper chains
    s4 = SceneBuilder()
    m4 = s4.lambertian(s4.solid((1, 1, 1)))
    b = s4.hlist([s4.translate(s4.box((0, 0, 0), (1, 1, 1), m4), (1, 0, 0)),
                  s4.translate(s4.box((0, 0, 0), (1, 1, 1), m4), (3, 0, 0))])
    st, _, msg = abi.scene_check(s4.desc(s4.volume(b, 0.1, s4.solid((1, 1, 1)))))
    assert st == abi.RT_ERR_UNSUPPORTED and "volume boundary" in msg


def test_big_scene_gets_a_bvh_within_the_stack():
    import random
    rnd = random.Random(3)
    s = SceneBuilder()
    m = s.lambertian(s.solid((0.5, 0.5, 0.5)))
    tris = []
    for _ in range(20000):
        c = [rnd.uniform(-50, 50) for _ in range(3)]
        tris.append(s.triangle(c, [c[0] + rnd.random(), c[1], c[2]], [c[0], c[1] + rnd.random(), c[2]], m))
    st, info, msg = abi.scene_check(s.desc(s.bvh(tris)))
    assert st == abi.RT_OK, msg
    assert info.triangles == 20000 and info.linear_ops == 0 and info.stack_need <= 32


def test_multi_create_without_device_fails_cleanly():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    lib = abi.load()
    h = ctypes.c_void_p()
    devs = (ctypes.c_int32 * 2)(0, 1)
    assert lib.rt_multi_create(devs, 2, ctypes.byref(h)) == abi.RT_ERR_NO_DEVICE
    assert not h.value and b"device" in lib.rt_multi_last_error(None)
