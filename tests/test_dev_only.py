"""A development build that instantiates one kernel family (RT_DEV_ONLY, scripts/dev_usage.sh) must refuse a
scene that needs another family with RT_ERR_UNSUPPORTED -- rt_scene_check on the host, and render() before it
launches anything -- instead of rendering black (round-4 verdict: an RT_DEV_ONLY build rendered a black
volume image). Builds the flat-only library with hipcc (gfx950 cross-compile, no GPU needed) and asks
rt_scene_check about a flat scene and a wide-BVH scene in a child process bound to that library."""
import hashlib
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


SRCS = ("rt_kernels.hip", "rt_multi.hip", "scene_compile.cpp", "rt_device.h", "rt_scene.h", "rt_sin.h",
        "scene_compile.h")


def dev_build():
    """The flat-only library, built once per source state (cached under build/dev_cache by the sources' hash,
    so a later CPU run does not pay the ~1-minute hipcc build again)."""
    h = hashlib.sha256()
    for f in SRCS + ("../../include/rt_hip.h",):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    cache = os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "build", "dev_cache")
    lib = os.path.join(cache, f"librt_hip_dev1_{h.hexdigest()[:16]}.so")
    if not os.path.exists(lib):
        os.makedirs(cache, exist_ok=True)
        for old in os.listdir(cache):  # older source states
            os.remove(os.path.join(cache, old))
        tmp = lib + ".tmp"
        cmd = [HIPCC, "-O1", "-std=c++17", "-fPIC", "-ffp-contract=on", "-fno-slp-vectorize", "--offload-arch=gfx950",
               "-DRT_DEV_ONLY=1", "-shared", "-o", tmp] + [os.path.join(CSRC, f) for f in SRCS[:3]] + ["-ldl"]
        subprocess.run(cmd, check=True, timeout=600)
        os.replace(tmp, lib)
    return lib


def child_env(lib):
    return dict(os.environ, RT_HIP_LIB=lib, PYTHONPATH=os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))


@pytest.mark.slow
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_dev_only_build_refuses_other_families():
    r = subprocess.run([sys.executable, "-c", CHILD], env=child_env(dev_build()), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.slow
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_gpu_session_on_a_dev_only_build_stops_at_collection():
    # round 5's red test_gpu_wide.py run: the GPU tests on a one-family development variant. The
    # library says what it is (rt_build_info), and tests/conftest.py ends such a session before any test runs.
    lib = dev_build()
    r = subprocess.run([sys.executable, "-c", "from rt_amd import abi; print(abi.build_info())"], env=child_env(lib),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "'dev_only': '1'" in r.stdout, r.stdout + r.stderr
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "gpu", "--collect-only", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "test_gpu_wide.py")], env=child_env(lib), cwd=REPO,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 4 and "development build" in r.stdout + r.stderr, r.stdout + r.stderr


def test_product_library_reports_its_configuration():
    from rt_amd import abi
    info = abi.build_info()
    assert info["dev_only"] == "0", info
    assert int(info["wide_top_n"]) > 0 and int(info["wide_lds_stack"]) > 0, info
