"""glTF 2.0 writer and the synthetic Sponza stand-ins.

The reference's C4 workload renders Sponza (main.cc:439-498) from
./assets/Sponza/glTF/Sponza.gltf. The reference ships that file but not its
Sponza.bin (9,528,220 bytes of vertex and index data), and there is no network here.

`write_sponza_standin` keeps the real Sponza.gltf (a copy of the reference's file is
under tests/golden/assets/Sponza/glTF) and writes a Sponza.bin that fills its layout:
the same 103 primitives of the last mesh, the same accessors, offsets and uint16 index
buffers (shared between primitives where the real file shares them), 262,267 triangles.
Each primitive's vertices form a planar grid spanning the two largest extents of its
accessor's min/max box at the box's centre, so the geometry sits where Sponza's objects
sit, with their triangle counts. Cells are split along one diagonal, then (only when a
primitive has more triangles than cells) along the other: coplanar duplicates shade
identically, so exact-t ties between them do not change an image.

`write_atrium_standin` is the earlier procedural atrium (floor, walls, gallery, columns).
"""
import json
import math
import os

import numpy as np

SPONZA_TRIANGLES = 262_267


def write_gltf(path, meshes, extra_buffers=0):
    """meshes: list of meshes, each a list of primitives: dict(positions=(n,3) float32,
    indices=uint16/uint32 array or None, stride=None|int, mode=4). All data goes into
    buffers[0] (<name>.bin next to the .gltf); `extra_buffers` adds unused buffers."""
    binpath = os.path.splitext(path)[0] + ".bin"
    blob = bytearray()
    views, accessors, gmeshes = [], [], []

    def add(arr, comp_type, typ, stride=None):
        while len(blob) % 4:
            blob.append(0)
        off = len(blob)
        blob.extend(arr.tobytes())
        view = {"buffer": 0, "byteOffset": off, "byteLength": arr.nbytes}
        if stride is not None:
            view["byteStride"] = stride
        views.append(view)
        count = arr.shape[0] if arr.ndim > 1 or typ == "SCALAR" else arr.size
        accessors.append({"bufferView": len(views) - 1, "componentType": comp_type, "count": int(count), "type": typ})
        return len(accessors) - 1

    for mesh in meshes:
        prims = []
        for pr in mesh:
            pos = np.ascontiguousarray(pr["positions"], dtype=np.float32).reshape(-1, 3)
            p = {"attributes": {"POSITION": add(pos, 5126, "VEC3", pr.get("stride"))}, "mode": pr.get("mode", 4)}
            idx = pr.get("indices")
            if idx is not None:
                idx = np.ascontiguousarray(idx)
                p["indices"] = add(idx.reshape(-1), 5123 if idx.dtype == np.uint16 else 5125, "SCALAR")
            prims.append(p)
        gmeshes.append({"primitives": prims})
    doc = {"asset": {"version": "2.0", "generator": "rt_amd.synth_gltf"},
           "buffers": [{"uri": os.path.basename(binpath), "byteLength": len(blob)}] +
                      [{"uri": "unused%d.bin" % k, "byteLength": 0} for k in range(extra_buffers)],
           "bufferViews": views, "accessors": accessors, "meshes": gmeshes,
           "nodes": [{"mesh": k} for k in range(len(gmeshes))], "scenes": [{"nodes": list(range(len(gmeshes)))}],
           "scene": 0}
    with open(binpath, "wb") as f:
        f.write(bytes(blob))
    with open(path, "w") as f:
        json.dump(doc, f)
    return path


def _grid(p0, u, v, nu, nv):
    """A (nu x nv)-cell parallelogram p0 + s u + t v as 2 nu nv triangles: (vertices, triangles)."""
    s = np.linspace(0.0, 1.0, nu + 1)
    t = np.linspace(0.0, 1.0, nv + 1)
    S, T = np.meshgrid(s, t, indexing="ij")
    verts = np.asarray(p0)[None, None, :] + S[..., None] * np.asarray(u) + T[..., None] * np.asarray(v)
    verts = verts.reshape(-1, 3)
    k = lambda i, j: i * (nv + 1) + j
    I, J = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    a, b, c, d = k(I, J), k(I + 1, J), k(I + 1, J + 1), k(I, J + 1)
    tris = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    return verts, tris


def _cylinder(center, radius, height, nseg, nring):
    ang = np.linspace(0.0, 2 * math.pi, nseg + 1)[:-1]
    y = np.linspace(0.0, height, nring + 1)
    A, Y = np.meshgrid(ang, y, indexing="ij")
    verts = np.stack([center[0] + radius * np.cos(A), center[1] + Y, center[2] + radius * np.sin(A)], -1).reshape(-1, 3)
    k = lambda i, j: (i % nseg) * (nring + 1) + j
    I, J = np.meshgrid(np.arange(nseg), np.arange(nring), indexing="ij")
    a, b, c, d = k(I, J), k(I + 1, J), k(I + 1, J + 1), k(I, J + 1)
    tris = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    return verts, tris


def sponza_standin_pieces():
    """(vertices, triangles) pieces of the atrium; 262,267 triangles in total."""
    pieces = []
    # two rows of 12 columns (r 45, 820 high, 48 x 40 quads each: 3,840 triangles; 92,160)
    for z in (-330.0, 330.0):
        for k in range(12):
            pieces.append(_cylinder((-1320.0 + 240.0 * k, 0.0, z), 45.0, 820.0, 48, 40))
    # side walls z = +-620, 0..1100 high (128 x 100 cells: 25,600 each; 51,200)
    for z, u in ((-620.0, (2900.0, 0, 0)), (620.0, (-2900.0, 0, 0))):
        x0 = -1450.0 if z < 0 else 1450.0
        pieces.append(_grid((x0, 0.0, z), u, (0, 1100.0, 0), 128, 100))
    # gallery floors at y = 430 between the columns and the walls (2 x 100 x 60 cells: 24,000)
    for z0, dz in ((-620.0, 290.0), (330.0, 290.0)):
        pieces.append(_grid((-1450.0, 430.0, z0), (2900.0, 0, 0), (0, 0, dz), 100, 60))
    # end walls x = +-1450 (2 x 60 x 50 cells: 12,000)
    for x, v in ((-1450.0, (0, 0, 1240.0)), (1450.0, (0, 0, -1240.0))):
        z0 = -620.0 if x < 0 else 620.0
        pieces.append(_grid((x, 0.0, z0), (0, 1100.0, 0), v, 60, 50))
    used = sum(len(t) for _, t in pieces)
    # the floor takes the rest: nu x nv cells (2 nu nv triangles) plus one triangle if odd
    rest = SPONZA_TRIANGLES - used
    nu, nv = min(((rest // (2 * b), b) for b in range(120, 200)), key=lambda c: rest - 2 * c[0] * c[1])
    pieces.append(_grid((-1450.0, 0.0, -620.0), (2900.0, 0, 0), (0, 0, 1240.0), nu, nv))
    left = SPONZA_TRIANGLES - used - 2 * nu * nv
    for i in range(left // 2):  # pairs of small floor tiles by the light's footprint
        pieces.append(_grid((10.0 + 20.0 * i, 0.5, 10.0), (15.0, 0, 0), (0, 0, 15.0), 1, 1))
    if left % 2:
        pieces.append((np.array([[0.0, 1.0, 0.0], [30.0, 1.0, 0.0], [0.0, 1.0, 30.0]]), np.array([[0, 1, 2]])))
    return pieces


SPONZA_LAYOUT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))),
                             "tests", "golden", "assets", "Sponza", "glTF", "Sponza.gltf")


def _layout_grid(nv, ntri):
    """(nx, ny, triangles (ntri, 3)) of a planar nx x ny grid with nx * ny <= nv vertices."""
    nx = max(2, int(math.isqrt(nv)))
    ny = max(2, nv // nx)
    while nx * ny > nv and ny > 2:
        ny -= 1
    if nx * ny > nv:
        raise ValueError(f"a primitive of {nv} vertices is too small for a grid")
    I, J = np.meshgrid(np.arange(nx - 1), np.arange(ny - 1), indexing="ij")
    a, b = I * ny + J, (I + 1) * ny + J
    c, d = b + 1, a + 1
    first = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    second = np.concatenate([np.stack([a, b, d], -1).reshape(-1, 3), np.stack([b, c, d], -1).reshape(-1, 3)])
    tris = np.concatenate([first, second])
    if ntri > len(tris):
        raise ValueError(f"{ntri} triangles do not fit a grid of {nv} vertices")
    return nx, ny, tris[:ntri]


def write_sponza_standin(directory, layout=SPONZA_LAYOUT):
    """Writes <directory>/Sponza.gltf (the real file) + a Sponza.bin filling its layout; returns the .gltf path.
    Without the layout file, the procedural atrium."""
    if not os.path.exists(layout):
        return write_atrium_standin(directory)
    os.makedirs(directory, exist_ok=True)
    with open(layout) as f:
        doc = json.load(f)
    acc, views = doc["accessors"], doc["bufferViews"]
    buf = np.zeros(doc["buffers"][0]["byteLength"], np.uint8)

    def span(a, elem):
        v = views[acc[a]["bufferView"]]
        off = v.get("byteOffset", 0) + acc[a].get("byteOffset", 0)
        return off, acc[a]["count"], elem

    prims = doc["meshes"][-1]["primitives"]  # the loader keeps the last mesh (gltf_loader.h:300-302)
    groups = {}  # index span -> primitives sharing it
    for p in prims:
        groups.setdefault(span(p["indices"], 2)[:2], []).append(p)
    for (ioff, icount), members in groups.items():
        nv = min(acc[p["attributes"]["POSITION"]]["count"] for p in members)
        nx, ny, tris = _layout_grid(nv, icount // 3)
        idx = np.zeros(icount, np.uint16)
        idx[: 3 * len(tris)] = tris.reshape(-1)
        buf[ioff: ioff + 2 * icount] = np.frombuffer(idx.tobytes(), np.uint8)
        for p in members:
            pa = p["attributes"]["POSITION"]
            lo, hi = np.array(acc[pa]["min"], float), np.array(acc[pa]["max"], float)
            ext = hi - lo
            u_ax, v_ax = [int(k) for k in np.argsort(-ext)[:2]]
            s = np.linspace(0.0, 1.0, nx)
            t = np.linspace(0.0, 1.0, ny)
            S, T = np.meshgrid(s, t, indexing="ij")
            pos = np.tile((lo + hi) / 2, (acc[pa]["count"], 1))
            g = np.tile((lo + hi) / 2, (nx * ny, 1))
            g[:, u_ax] = lo[u_ax] + S.reshape(-1) * ext[u_ax]
            g[:, v_ax] = lo[v_ax] + T.reshape(-1) * ext[v_ax]
            pos[: nx * ny] = g
            poff, pcount, _ = span(pa, 12)
            buf[poff: poff + 12 * pcount] = np.frombuffer(pos.astype(np.float32).tobytes(), np.uint8)
    with open(os.path.join(directory, doc["buffers"][0]["uri"]), "wb") as f:
        f.write(buf.tobytes())
    path = os.path.join(directory, "Sponza.gltf")
    with open(path, "w") as f:
        json.dump(doc, f)
    return path


def write_atrium_standin(directory):
    """Writes <directory>/Sponza.gltf + Sponza.bin (the procedural atrium); returns the .gltf path."""
    os.makedirs(directory, exist_ok=True)
    prims, verts, tris = [], [], []

    def flush():
        if tris:
            prims.append({"positions": np.concatenate(verts).astype(np.float32),
                          "indices": np.concatenate(tris).astype(np.uint16)})
            verts.clear()
            tris.clear()

    nvert = 0
    for v, t in sponza_standin_pieces():
        if nvert + len(v) > 65535:
            flush()
            nvert = 0
        verts.append(v)
        tris.append(t + nvert)
        nvert += len(v)
    flush()
    decoy = [{"positions": np.zeros((3, 3), np.float32), "indices": None}]  # not the last mesh: ignored
    return write_gltf(os.path.join(directory, "Sponza.gltf"), [decoy, prims])
