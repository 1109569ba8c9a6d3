#!/usr/bin/env python3
"""How closed is a config scene's triangle mesh? Counts, over the triangles of the scene descriptor the C++ plugin
surface builds (rt_amd.plugin.ConfigScene), the edges used by one triangle (a boundary: a ray near it passes into a
hole on one side, so an fp32 edge decision there can change the path) and by two (shared: either triangle's hit is
the same surface). Round 6: the C4 stand-in (rt_amd.synth_gltf) is a sieve -- the real Sponza.gltf's index triples
over grid-placed vertices -- which is what its fp32 divergence comes from.

    python scripts/dev_mesh_edges.py [scene] [width]        (default: sponza_lit 320; CPU only)"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))
import bench  # noqa: E402
from rt_amd import abi, plugin  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "sponza_lit"
    width = int(sys.argv[2]) if len(sys.argv) > 2 else 320
    if name.startswith("sponza"):
        bench.sponza_asset()
    cs = plugin.ConfigScene(name, width, 16.0 / 9.0)
    d = cs.desc
    tris = [[[o.a[j] for j in range(3)], [o.b[j] for j in range(3)], [o.c[j] for j in range(3)]]
            for o in (d.objects[i] for i in range(d.num_objects)) if o.kind == abi.RT_OBJ_TRIANGLE]
    T = np.array(tris, dtype=np.float64)
    _, inv = np.unique(np.round(T.reshape(-1, 3), 5), axis=0, return_inverse=True)
    F = inv.reshape(-1, 3)
    E = np.sort(np.concatenate([F[:, [0, 1]], F[:, [1, 2]], F[:, [2, 0]]]), axis=1)
    _, cnt = np.unique(E, axis=0, return_counts=True)
    once, twice, more = int((cnt == 1).sum()), int((cnt == 2).sum()), int((cnt > 2).sum())
    print(f"{name}: {len(F)} triangles, {len(cnt)} distinct edges: {once} used by one triangle (boundary), {twice} by "
          f"two, {more} by more; {once / (3 * len(F)):.3f} of the triangles' edges are on a boundary")


if __name__ == "__main__":
    main()
