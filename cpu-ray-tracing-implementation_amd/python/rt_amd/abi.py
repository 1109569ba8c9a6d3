"""ctypes mirror of include/rt_hip.h (the C ABI of librt_hip.so).

The structs below must match include/rt_hip.h byte for byte;
tests/test_boundary.py checks their sizes against the C compiler's.
"""
import ctypes
import os

c_int32, c_uint32, c_uint64, c_double, c_float = (ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64,
                                                  ctypes.c_double, ctypes.c_float)
D3 = c_double * 3

PKG_DIR = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REPO_DIR = os.path.dirname(PKG_DIR)
BUILD_DIR = os.path.join(PKG_DIR, "build")

# rt_status
RT_OK, RT_ERR_INVALID_ARGUMENT, RT_ERR_UNSUPPORTED, RT_ERR_HIP, RT_ERR_OUT_OF_MEMORY, RT_ERR_NO_SCENE, \
    RT_ERR_NO_DEVICE = range(7)
# rt_object_kind
RT_OBJ_SPHERE, RT_OBJ_QUAD, RT_OBJ_TRIANGLE, RT_OBJ_LIST, RT_OBJ_BVH, RT_OBJ_TRANSLATE, RT_OBJ_ROTATE_X, \
    RT_OBJ_ROTATE_Y, RT_OBJ_ROTATE_Z, RT_OBJ_VOLUME = range(1, 11)
# rt_material_kind
RT_MAT_LAMBERTIAN, RT_MAT_METAL, RT_MAT_DIELECTRIC, RT_MAT_ISOTROPIC, RT_MAT_DIFFUSE_LIGHT, RT_MAT_GLOSS = range(1, 7)
RT_TEX_SOLID, RT_TEX_CHECKER, RT_TEX_PERLIN, RT_TEX_VALUE, RT_TEX_WORLEY, RT_TEX_VORONOI, RT_TEX_IMAGE = range(1, 8)
RT_CAM_PERSPECTIVE, RT_CAM_ORTHONORMAL, RT_CAM_FISHEYE, RT_CAM_LENS = range(4)
RT_PREC_F32, RT_PREC_F64 = 0, 1
RT_TRAV_AUTO, RT_TRAV_ORDERED = 0, 1
ABI_VERSION = 8  # include/rt_hip.h RT_ABI_VERSION


class rt_object(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("material", c_int32), ("child", c_int32), ("first_child", c_int32),
                ("child_count", c_int32), ("moving", c_int32), ("a", D3), ("b", D3), ("c", D3), ("s0", c_double),
                ("s1", c_double)]


class rt_material(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("texture", c_int32), ("fuzz", c_float), ("refraction", c_float),
                ("smoothness", c_float), ("specular_prob", c_float)]


class rt_texture(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("data", c_int32), ("color", D3), ("odd", D3), ("even", D3), ("scale", c_double)]


class rt_scene_desc(ctypes.Structure):
    _fields_ = [("objects", ctypes.POINTER(rt_object)), ("num_objects", c_int32),
                ("children", ctypes.POINTER(c_int32)), ("num_children", c_int32),
                ("materials", ctypes.POINTER(rt_material)), ("num_materials", c_int32),
                ("textures", ctypes.POINTER(rt_texture)), ("num_textures", c_int32),
                ("world", c_int32), ("light", c_int32), ("background", c_int32), ("pad_", c_int32),
                ("tex_data", ctypes.POINTER(c_double)), ("num_tex_data", ctypes.c_int64),
                ("image_data", ctypes.POINTER(ctypes.c_uint8)), ("num_image_data", ctypes.c_int64)]


class rt_camera_desc(ctypes.Structure):
    _fields_ = [("mode", c_int32), ("image_width", c_int32), ("image_height", c_int32), ("pad_", c_int32),
                ("pos", D3), ("dir", D3), ("right", D3), ("up", D3), ("viewport_width", c_double),
                ("viewport_height", c_double), ("focal_length", c_double), ("focus_dist", c_double),
                ("defocus_u", D3), ("defocus_v", D3)]


class rt_render_params(ctypes.Structure):
    _fields_ = [("spp", c_int32), ("max_depth", c_int32), ("seed", c_uint64), ("precision", c_int32),
                ("first_sample", c_int32), ("samples_per_item", c_int32), ("pool_slots", c_int32),
                ("segments_per_launch", c_int32), ("traversal", c_int32)]


class rt_tile(ctypes.Structure):
    _fields_ = [("x0", c_int32), ("y0", c_int32), ("width", c_int32), ("height", c_int32)]


class rt_counters(ctypes.Structure):
    _fields_ = [("segments", c_uint64), ("samples", c_uint64), ("iterations", c_uint64), ("launches", c_uint64),
                ("last_render_ms", c_double), ("step_ms", c_double), ("aux_ms", c_double),
                ("grid_lanes", c_uint64), ("passes", c_uint64), ("partial_bytes", c_uint64)]


class rt_scene_info(ctypes.Structure):
    _fields_ = [("quads", c_int32), ("spheres", c_int32), ("triangles", c_int32), ("instances", c_int32),
                ("volumes", c_int32), ("bvh_nodes", c_int32), ("linear_ops", c_int32), ("stack_need", c_int32),
                ("bytes_f32", c_uint64), ("bytes_f64", c_uint64), ("flat_quads", c_int32), ("flat_boxes", c_int32),
                ("wide_nodes", c_int32), ("wide_stack", c_int32), ("wide_kinds", c_int32), ("wide_prim_words", c_int32),
                ("wide_big", c_int32)]


# every symbol include/rt_hip.h declares, with its ctypes signature
SIGNATURES = {
    "rt_abi_version": (c_int32, []),
    "rt_build_info": (ctypes.c_char_p, []),
    "rt_context_create": (c_int32, [c_int32, ctypes.POINTER(ctypes.c_void_p)]),
    "rt_context_destroy": (None, [ctypes.c_void_p]),
    "rt_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "rt_scene_upload": (c_int32, [ctypes.c_void_p, ctypes.POINTER(rt_scene_desc)]),
    "rt_scene_check": (c_int32, [ctypes.POINTER(rt_scene_desc), ctypes.POINTER(rt_scene_info), ctypes.c_char_p,
                                 c_int32]),
    "rt_render_tiles": (c_int32, [ctypes.c_void_p, ctypes.POINTER(rt_camera_desc), ctypes.POINTER(rt_render_params),
                                  ctypes.POINTER(rt_tile), c_int32, ctypes.c_void_p, c_int32, ctypes.c_void_p]),
    "rt_stats": (c_int32, [ctypes.c_void_p, ctypes.POINTER(rt_counters)]),
    "rt_reset_counters": (c_int32, [ctypes.c_void_p]),
    "rt_set_timing": (c_int32, [ctypes.c_void_p, c_int32]),
    "rt_rng_u32": (c_uint32, [c_uint64, c_uint32, c_uint32, c_uint32]),
    "rt_multi_create": (c_int32, [ctypes.POINTER(c_int32), c_int32, ctypes.POINTER(ctypes.c_void_p)]),
    "rt_multi_destroy": (None, [ctypes.c_void_p]),
    "rt_multi_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "rt_multi_uses_rccl": (c_int32, [ctypes.c_void_p]),
    "rt_multi_scene_upload": (c_int32, [ctypes.c_void_p, ctypes.POINTER(rt_scene_desc)]),
    "rt_multi_render": (c_int32, [ctypes.c_void_p, ctypes.POINTER(rt_camera_desc), ctypes.POINTER(rt_render_params),
                                  c_int32, ctypes.c_void_p]),
    "rt_multi_stats": (c_int32, [ctypes.c_void_p, c_int32, ctypes.POINTER(rt_counters)]),
    "rt_multi_plan": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_int32, ctypes.POINTER(rt_tile), c_int32]),
    "rt_multi_comm_inits": (c_uint64, []),
}


class TileList:
    """A tile list as the ctypes array rt_render_tiles takes, built once: a caller that renders the same
    tiles every frame (rt_amd.distributed.FrameSharding) passes this instead of a list, whose conversion
    (one rt_tile per 16x16 tile: C1's 625, C2's 2,500) costs ~1 us of Python per tile and call."""

    def __init__(self, tiles):
        self.tiles = [tuple(t) for t in tiles]
        self.n = len(self.tiles)
        self.arr = (rt_tile * max(1, self.n))(*[rt_tile(*t) for t in self.tiles])

    def __len__(self):
        return self.n

    def __iter__(self):
        return iter(self.tiles)


_lib = None


def lib_path():
    # RT_HIP_LIB: a development build of the same library (scripts/build_variant.sh)
    return os.environ.get("RT_HIP_LIB") or os.path.join(BUILD_DIR, "librt_hip.so")


def load():
    """Load librt_hip.so (built in-tree by __graft_entry__.build()). Fails loudly if missing."""
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        # One HIP runtime per process: librt_hip needs libamdhip64.so.7, and so does PyTorch, which bundles its
        # own. Loaded first, librt_hip would bring in /opt/rocm's, and a later `import torch` would bind to that
        # one and find no GPU ("No HIP GPUs are available"). PyTorch first, librt_hip then binds to its runtime.
        # (plugin.load goes through here too: librt_scenes links librt_hip.)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.rt_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{path} has ABI {lib.rt_abi_version()}, this binding expects {ABI_VERSION}: rebuild")
        _lib = lib
    return _lib


def build_info():
    """The library's compile-time configuration (rt_build_info): {"dev_only": "0", "wide_top_n": "55", ...}."""
    return dict(w.split("=", 1) for w in load().rt_build_info().decode().split())


def scene_check(desc):
    """Compile a descriptor on the host (no GPU). Returns (status, rt_scene_info, message)."""
    info = rt_scene_info()
    err = ctypes.create_string_buffer(512)
    st = load().rt_scene_check(ctypes.byref(desc), ctypes.byref(info), err, 512)
    return st, info, err.value.decode()


class RTError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"rt status {status}: {msg}")
        self.status = status
