"""Config scenes start from a process-fresh rand() state (main.cc:633-690 builds one scene per process).

The scenes that draw from glibc's rand() -- the perlin and value tables (noise.h:10-136), the box
heights of perlin_texture_ball (main.cc:402-437), the RTOW spheres (main.cc:105-153) -- must give
the same descriptor whether they are built first or after other scenes in the same process.
"""
import ctypes

import pytest

from rt_amd import plugin

DRAWING = ["perlin_texture_ball", "test_perlin_noise", "test_value_noise", "rtow"]


def desc_bytes(cs):
    """Every byte the descriptor points to (objects, children, materials, textures, tables, images)."""
    d = cs.desc

    def arr(ptr, n, ty):
        return bytes((ty * n).from_address(ctypes.addressof(ptr.contents))) if n > 0 else b""

    return b"|".join([
        arr(d.objects, d.num_objects, type(d.objects.contents)),
        arr(d.children, d.num_children, ctypes.c_int32),
        arr(d.materials, d.num_materials, type(d.materials.contents)),
        arr(d.textures, d.num_textures, type(d.textures.contents)),
        arr(d.tex_data, d.num_tex_data, ctypes.c_double),
        arr(d.image_data, d.num_image_data, ctypes.c_uint8),
        bytes(f"{d.world} {d.light} {d.background}", "ascii"),
    ])


@pytest.mark.parametrize("name", DRAWING)
def test_scene_independent_of_build_order(name):
    first = desc_bytes(plugin.ConfigScene(name, 40))
    # scenes that draw from rand() built before it in the same process
    for other in DRAWING + ["cornell_box"]:
        plugin.ConfigScene(other, 40)
    again = desc_bytes(plugin.ConfigScene(name, 40))
    assert first == again, name
