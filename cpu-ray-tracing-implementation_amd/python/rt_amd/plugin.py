"""The C++ plugin surface (../../rt/*.h) as built into librt_scenes.so: the
reference's main.cc config scenes assembled with camera / hittable / material
objects, flattened exactly as camera::render flattens them."""
import ctypes
import os

from . import abi

_lib = None


def load():
    global _lib
    if _lib is None:
        path = os.path.join(abi.BUILD_DIR, "librt_scenes.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: run `make`")
        abi.load()  # librt_scenes links librt_hip: loaded the way abi.load does (PyTorch's HIP runtime first)
        L = ctypes.CDLL(path)
        P = ctypes.POINTER
        L.rtsc_build.restype = ctypes.c_void_p
        L.rtsc_build.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_double, P(abi.rt_scene_desc),
                                 P(abi.rt_camera_desc), P(ctypes.c_int), P(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
        L.rtsc_free.argtypes = [ctypes.c_void_p]
        L.rtsc_gltf_triangles.restype = ctypes.c_longlong
        L.rtsc_gltf_triangles.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_char_p,
                                          ctypes.c_int]
        L.rtsc_render_ppm_on.restype = ctypes.c_int
        L.rtsc_render_ppm_on.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                                         ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.rtsc_render_ppm_repeat.restype = ctypes.c_int
        L.rtsc_render_ppm_repeat.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.c_int,
                                             ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.rtsc_render_ppm.restype = ctypes.c_int
        L.rtsc_render_ppm.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        _lib = L
    return _lib


class ConfigScene:
    """desc / cam / spp / max_depth of a main.cc scene built by the C++ plugin surface."""

    def __init__(self, name, width=0, aspect=0.0):
        L = load()
        self.desc, self.cam = abi.rt_scene_desc(), abi.rt_camera_desc()
        spp, depth = ctypes.c_int(), ctypes.c_int()
        err = ctypes.create_string_buffer(256)
        self._h = L.rtsc_build(name.encode(), width, aspect, ctypes.byref(self.desc), ctypes.byref(self.cam),
                               ctypes.byref(spp), ctypes.byref(depth), err, 256)
        if not self._h:
            raise RuntimeError(f"rtsc_build({name}): {err.value.decode()}")
        self.spp, self.max_depth = spp.value, depth.value
        self.desc._owner = self  # the descriptor points into memory this handle owns

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.rtsc_free(self._h)
            self._h = None


def render_ppm(name, path, width=0, aspect=0.0, spp=0, max_depth=0, seed=1, precision=abi.RT_PREC_F32, devices=None,
               repeat=1):
    """camera::render(of, world, light) of a config scene into a PPM file (the whole drop-in path);
    devices: camera::devices_ (the image tiled over those GPUs through rt_multi_*); repeat: render that
    many times with the same camera object (it keeps its contexts / communicator between renders)."""
    err = ctypes.create_string_buffer(512)
    devs = list(devices or [])
    arr = (ctypes.c_int32 * max(1, len(devs)))(*devs)
    rc = load().rtsc_render_ppm_repeat(name.encode(), width, aspect, spp, max_depth, seed, precision, arr, len(devs),
                                       repeat, path.encode(), err, 512)
    if rc != 0:
        raise RuntimeError(f"camera::render failed: {err.value.decode()}")


def gltf_triangles(path):
    """The triangles main.cc's sponza() builds from a glTF file (gltf_loader.h quirks included),
    as an (n, 3, 3) float64 array."""
    import numpy as np
    L = load()
    err = ctypes.create_string_buffer(512)
    n = L.rtsc_gltf_triangles(path.encode(), None, 0, err, 512)
    if n < 0:
        raise RuntimeError(f"glTF load failed: {err.value.decode()}")
    out = np.zeros((max(n, 1), 3, 3), dtype=np.float64)
    L.rtsc_gltf_triangles(path.encode(), out.ctypes.data, n, err, 512)
    return out[:n]
