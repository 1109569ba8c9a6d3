"""glTF ingestion (rt/gltf_loader.h) and the triangles main.cc's sponza() builds from it
(main.cc:439-486), on small files written by rt_amd.synth_gltf. Each test names the
reference behaviour it pins (gltf_loader.h / main.cc line numbers)."""
import json
import os

import numpy as np
import pytest

from rt_amd import abi, plugin, synth_gltf

TRI = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
QUAD = np.array([[0, 0, 0], [2, 0, 0], [2, 2, 0], [0, 2, 0]], np.float32)


def write(tmp_path, meshes, name="m.gltf", **kw):
    return synth_gltf.write_gltf(str(tmp_path / name), meshes, **kw)


def test_indexed_primitive(tmp_path):
    p = write(tmp_path, [[{"positions": QUAD, "indices": np.array([0, 1, 2, 0, 2, 3], np.uint16)}]])
    t = plugin.gltf_triangles(p)
    assert t.shape == (2, 3, 3)
    np.testing.assert_array_equal(t[1], QUAD[[0, 2, 3]])


def test_only_the_last_mesh_is_kept(tmp_path):
    # gltf_loader.h:300-302: every mesh overwrites output_primitives_
    first = [{"positions": QUAD + 10, "indices": np.array([0, 1, 2], np.uint16)}]
    last = [{"positions": TRI, "indices": None}, {"positions": TRI + 5, "indices": None}]
    t = plugin.gltf_triangles(write(tmp_path, [first, last]))
    assert t.shape == (2, 3, 3)
    np.testing.assert_array_equal(t[0], TRI)
    np.testing.assert_array_equal(t[1], TRI + 5)


def test_non_indexed_primitive_takes_position_triples(tmp_path):
    # main.cc:479-484: without indices, positions (3k, 3k+1, 3k+2); a trailing partial triple is dropped
    pos = np.concatenate([TRI, TRI + 1, TRI[:2] + 2])
    t = plugin.gltf_triangles(write(tmp_path, [[{"positions": pos, "indices": None}]]))
    assert t.shape == (2, 3, 3)
    np.testing.assert_array_equal(t[1], TRI + 1)


def test_uint32_indices_give_no_triangles(tmp_path):
    # main.cc:461-469 reads only unsigned-short indices; use_indices stays true, so nothing is drawn
    p = write(tmp_path, [[{"positions": QUAD, "indices": np.array([0, 1, 2], np.uint32)},
                          {"positions": TRI, "indices": np.array([0, 1, 2], np.uint16)}]])
    t = plugin.gltf_triangles(p)
    assert t.shape == (1, 3, 3)
    np.testing.assert_array_equal(t[0], TRI)


def test_byte_stride_does_not_deinterleave(tmp_path):
    # gltf_loader.h:662-672: the copy is contiguous whatever byteStride says (default 1)
    p = write(tmp_path, [[{"positions": QUAD, "indices": np.array([0, 1, 2], np.uint16), "stride": 12}]])
    np.testing.assert_array_equal(plugin.gltf_triangles(p)[0], QUAD[:3])
    p2 = write(tmp_path, [[{"positions": QUAD, "indices": np.array([1, 2, 3], np.uint16), "stride": 24}]], "s.gltf")
    np.testing.assert_array_equal(plugin.gltf_triangles(p2)[0], QUAD[1:])


def test_only_buffers0_is_read(tmp_path):
    # gltf_loader.h:565: buffers[0].uri; further buffers are never opened
    p = write(tmp_path, [[{"positions": TRI, "indices": None}]], extra_buffers=2)
    assert not os.path.exists(tmp_path / "unused0.bin")
    assert plugin.gltf_triangles(p).shape == (1, 3, 3)


def test_non_float_positions_are_skipped(tmp_path):
    # main.cc:451-460: only float positions are converted
    p = write(tmp_path, [[{"positions": TRI, "indices": None}]])
    doc = json.load(open(p))
    doc["accessors"][0]["componentType"] = 5123  # unsigned short positions
    doc["accessors"][0]["count"] = 1
    json.dump(doc, open(p, "w"))
    assert plugin.gltf_triangles(p).shape == (0, 3, 3)


@pytest.mark.parametrize("mutate,msg", [
    (lambda d: d["buffers"][0].update(uri="missing.bin"), "cannot open"),
    (lambda d: d["accessors"][0].update(count=1000), "past the end"),
    (lambda d: d["accessors"][0].update(type="VEC7"), "accessor type"),
    (lambda d: d["accessors"][0].update(componentType=9999), "component type"),
    (lambda d: d["meshes"][0]["primitives"][0].update(mode=9), "primitive mode"),
    (lambda d: d["buffers"][0].pop("uri"), "uri"),
])
def test_errors(tmp_path, mutate, msg):
    p = write(tmp_path, [[{"positions": TRI, "indices": None}]])
    doc = json.load(open(p))
    mutate(doc)
    json.dump(doc, open(p, "w"))
    with pytest.raises(RuntimeError, match=msg):
        plugin.gltf_triangles(p)


def test_json_syntax(tmp_path):
    p = write(tmp_path, [[{"positions": TRI, "indices": None}]])
    text = open(p).read()
    # whitespace, escapes and nesting the reader must accept
    doc = json.loads(text)
    doc["asset"]["copyright"] = "café \"q\" \\ ☺ \U0001F600"
    doc["extras"] = {"a": [1, -2.5e-3, True, False, None, {"b": []}]}
    open(p, "w").write(json.dumps(doc, indent=3, ensure_ascii=True))
    assert plugin.gltf_triangles(p).shape == (1, 3, 3)
    open(p, "w").write(text[:-5])  # truncated
    with pytest.raises(RuntimeError, match="json"):
        plugin.gltf_triangles(p)


def test_path_without_directory_looks_at_the_root(tmp_path, monkeypatch):
    # gltf_loader.h:567-568: dir = path up to the last '/', then dir + "/" + uri -- with no '/'
    # in the path the buffer is looked up at /<uri>, as in the reference
    write(tmp_path, [[{"positions": TRI, "indices": None}]], "rootquirk.gltf")
    monkeypatch.chdir(tmp_path)
    with pytest.raises(RuntimeError, match="/rootquirk.bin"):
        plugin.gltf_triangles("rootquirk.gltf")
    assert plugin.gltf_triangles("./rootquirk.gltf").shape == (1, 3, 3)


def test_sponza_standin_scene(tmp_path, monkeypatch):
    # main.cc:439-498 on the synthetic stand-in: 262,267 triangles + the light quad, one shared
    # material record after the compiler merges the per-triangle lambertians
    p = synth_gltf.write_sponza_standin(str(tmp_path))
    assert plugin.gltf_triangles(p).shape == (synth_gltf.SPONZA_TRIANGLES, 3, 3)
    monkeypatch.setenv("RT_SPONZA_GLTF", p)
    cs = plugin.ConfigScene("sponza")
    assert (cs.cam.image_width, cs.spp, cs.max_depth) == (200, 30, 5)
    assert cs.desc.light >= 0
    st, info, msg = abi.scene_check(cs.desc)
    assert st == abi.RT_OK, msg
    assert info.triangles == synth_gltf.SPONZA_TRIANGLES and info.quads == 1
    assert info.linear_ops == 0 and info.stack_need <= 32


def test_sponza_without_asset_fails_cleanly(monkeypatch, tmp_path):
    monkeypatch.setenv("RT_SPONZA_GLTF", str(tmp_path / "nope.gltf"))
    with pytest.raises(RuntimeError, match="cannot open"):
        plugin.ConfigScene("sponza")
