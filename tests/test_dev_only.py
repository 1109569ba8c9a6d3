"""A development build that instantiates one kernel family (RT_DEV_ONLY, scripts/dev_usage.sh) must refuse a
scene that needs another family with RT_ERR_UNSUPPORTED -- rt_scene_check on the host, and render() before it
launches anything -- instead of rendering black (round-4 verdict: an RT_DEV_ONLY build rendered a black
volume image). Builds the flat-only library with hipcc (gfx950 cross-compile, no GPU needed) and asks
rt_scene_check about a flat scene and a wide-BVH scene in a child process bound to that library."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

CHILD = r'''
import sys
from rt_amd import abi, scenes
for name, want in (("cornell_box", abi.RT_OK), ("rtow", abi.RT_ERR_UNSUPPORTED),
                   ("cornell_box_with_volume", abi.RT_ERR_UNSUPPORTED)):
    desc = scenes.SCENES[name](width=16)[0]
    st, info, msg = abi.scene_check(desc)
    print(name, st, msg)
    assert st == want, (name, st, msg)
    if st != abi.RT_OK:
        assert "RT_DEV_ONLY" in msg, msg
'''


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_dev_only_build_refuses_other_families(tmp_path):
    lib = str(tmp_path / "librt_hip_dev1.so")
    cmd = [HIPCC, "-O1", "-std=c++17", "-fPIC", "-ffp-contract=on", "-fno-slp-vectorize", "--offload-arch=gfx950",
           "-DRT_DEV_ONLY=1", "-shared", "-o", lib] + [os.path.join(CSRC, f) for f in
                                                      ("rt_kernels.hip", "rt_multi.hip", "scene_compile.cpp")] + ["-ldl"]
    subprocess.run(cmd, check=True, timeout=600)
    env = dict(os.environ, RT_HIP_LIB=lib,
               PYTHONPATH=os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
