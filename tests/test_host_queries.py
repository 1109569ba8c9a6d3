"""Host-side hittable queries of the drop-in plugin surface (hittable::hit, get_bounding_box,
pdf_value, random; reference src/hittable.h:32-41): tests/native/host_queries.cpp against
known answers. Rendering never uses them (the device traces every ray); they let code written
against the reference's classes ask a scene object a question on the host."""
import os
import subprocess

import pytest

from rt_amd import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "rt")


@pytest.fixture(scope="module")
def out(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("hq") / "host_queries")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "-I", RT, "-o",
                    exe, os.path.join(REPO, "tests", "native", "host_queries.cpp"), "-L", abi.BUILD_DIR, "-lrt_hip",
                    "-Wl,-rpath," + abi.BUILD_DIR], check=True)
    lines = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    return {ln.split()[0]: [float(x) for x in ln.split()[1:]] for ln in lines if ln}


def rec(out, name):
    h, t, px, py, pz, nx, ny, nz, front, u, v = out[name]
    return dict(hit=bool(h), t=t, p=(px, py, pz), n=(nx, ny, nz), front=bool(front), u=u, v=v)


def test_sphere(out):
    r = rec(out, "sphere")  # sphere.h:40-74, uv from sphere.h:90-95
    assert r["hit"] and r["t"] == 1.5 and r["p"] == (0, 0, -1.5) and r["n"] == (0, 0, 1) and r["front"]
    assert (r["u"], r["v"]) == (0.25, 0.5)
    r = rec(out, "sphere_inside")  # the far root, seen from inside: back face
    assert r["hit"] and r["t"] == 0.5 and r["n"] == (0, 0, 1) and not r["front"]
    assert not rec(out, "sphere_miss")["hit"]


def test_moving_sphere_keeps_the_reference_normal(out):
    # centre at time 0.5 is (0, 0.5, -2), but the normal is (p - center_) / r with center_ = 0 (sphere.h:69)
    r = rec(out, "moving")
    assert r["hit"] and r["t"] == 1.5 and r["p"] == (0, 0.5, -1.5) and r["n"] == (0, -1, 3) and not r["front"]


def test_quad_hit_pdf_and_random(out):
    r = rec(out, "quad")
    assert r["hit"] and r["t"] == 3 and (r["u"], r["v"]) == (0.5, 0.5) and r["n"] == (0, 0, 1)
    assert rec(out, "quad_edge")["hit"]  # interval(0, 1) is closed (quad.h:58-64)
    assert out["quad_pdf"] == [9.0, 0.0]  # t^2 |d|^2 / (|cos| area), 0 on a miss (quad.h:66-73)
    x, y, z = out["quad_random"]  # corner + r1 u + r2 v - origin, on the quad's plane
    assert z == -3 and -0.5 <= x <= 0.5 and -0.5 <= y <= 0.5


def test_triangle_leaves_uv(out):
    r = rec(out, "triangle")  # triangle.h:30-40 writes t, p, normal and mat only
    assert r["hit"] and r["t"] == 4 and r["n"] == (0, 0, 1) and (r["u"], r["v"]) == (7, 9)
    assert not rec(out, "triangle_miss")["hit"]


def test_instances(out):
    r = rec(out, "rotate_y")  # hittable.h:192-216: the +z quad turned to face +x
    assert r["hit"] and r["t"] == 3 and abs(r["p"][0]) < 1e-15 and r["n"][0] == 1 and abs(r["n"][2]) < 1e-15
    r = rec(out, "translate")  # hittable.h:75-82
    assert r["hit"] and r["t"] == 5 and r["p"] == (0.25, 0.25, -5)
    lo_x, hi_x, lo_z, hi_z = out["rotate_box"]  # thin box padded to 1e-4 (aabb.h:81-86)
    assert hi_x - lo_x == pytest.approx(1e-4) and (lo_z, hi_z) == (-0.5, 0.5)


def test_bvh_node_tree_agrees_with_the_list(out):
    agree, hits, n = out["bvh_vs_list"]
    assert agree == n and 0.2 * n < hits < n
    assert out["boxes_equal"] == [1.0]


def test_volume_draws_its_free_flight(out):
    r = rec(out, "volume_thick")  # volumne.h:18-46: density 1e9 scatters right at the boundary
    assert r["hit"] and r["t"] == pytest.approx(4, abs=1e-6) and r["n"] == (1, 0, 0) and r["front"]
    assert not rec(out, "volume_thin")["hit"]
