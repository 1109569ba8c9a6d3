"""Thin Python handle over the C ABI: one Context per HIP device."""
import ctypes

import numpy as np

from . import abi


class Context:
    def __init__(self, device=0):
        self.lib = abi.load()
        h = ctypes.c_void_p()
        st = self.lib.rt_context_create(device, ctypes.byref(h))
        if st != abi.RT_OK:
            raise abi.RTError(st, self.lib.rt_last_error(None).decode())
        self.h = h

    def close(self):
        if self.h:
            self.lib.rt_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        if st != abi.RT_OK:
            raise abi.RTError(st, self.lib.rt_last_error(self.h).decode())

    def upload(self, desc):
        self._check(self.lib.rt_scene_upload(self.h, ctypes.byref(desc)))

    def set_timing(self, on):
        self._check(self.lib.rt_set_timing(self.h, 1 if on else 0))

    def stats(self):
        c = abi.rt_counters()
        self._check(self.lib.rt_stats(self.h, ctypes.byref(c)))
        return c

    def reset_counters(self):
        self._check(self.lib.rt_reset_counters(self.h))

    @staticmethod
    def params(spp, max_depth, seed=1, precision=abi.RT_PREC_F32, first_sample=0, samples_per_item=0, pool_slots=0,
               segments_per_launch=0, traversal=0):
        return abi.rt_render_params(spp=spp, max_depth=max_depth, seed=seed, precision=precision,
                                    first_sample=first_sample, samples_per_item=samples_per_item,
                                    pool_slots=pool_slots, segments_per_launch=segments_per_launch,
                                    traversal=traversal)

    def render_tiles(self, cam, params, tiles, out_ptr, out_is_device, stream=None):
        """`tiles`: a list of (x, y, w, h), or an abi.TileList built once for tiles rendered every frame."""
        arr = tiles.arr if isinstance(tiles, abi.TileList) else abi.TileList(tiles).arr
        self._check(self.lib.rt_render_tiles(self.h, ctypes.byref(cam), ctypes.byref(params), arr, len(tiles),
                                             ctypes.c_void_p(out_ptr), int(out_is_device),
                                             ctypes.c_void_p(stream or 0)))

    def render(self, cam, spp, max_depth, seed=1, precision=abi.RT_PREC_F32, tiles=None, **kw):
        """Render to a host numpy array (H, W, 3) -- or the packed tiles, (npix, 3)."""
        p = self.params(spp, max_depth, seed, precision, **kw)
        full = tiles is None
        if full:
            tiles = [(0, 0, cam.image_width, cam.image_height)]
        npix = sum(t[2] * t[3] for t in tiles)
        out = np.zeros((npix, 3), dtype=np.float64 if precision == abi.RT_PREC_F64 else np.float32)
        self.render_tiles(cam, p, tiles, out.ctypes.data, 0)
        return out.reshape(cam.image_height, cam.image_width, 3) if full else out


class Multi:
    """rt_multi_*: one process driving several devices (tiles round-robin, RCCL gather to devices[0])."""

    def __init__(self, devices):
        self.lib = abi.load()
        arr = (ctypes.c_int32 * len(devices))(*devices)
        h = ctypes.c_void_p()
        st = self.lib.rt_multi_create(arr, len(devices), ctypes.byref(h))
        if st != abi.RT_OK:
            raise abi.RTError(st, self.lib.rt_multi_last_error(None).decode())
        self.h, self.n = h, len(devices)

    def close(self):
        if self.h:
            self.lib.rt_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st):
        if st != abi.RT_OK:
            raise abi.RTError(st, self.lib.rt_multi_last_error(self.h).decode())

    @property
    def uses_rccl(self):
        return bool(self.lib.rt_multi_uses_rccl(self.h))

    def upload(self, desc):
        self._check(self.lib.rt_multi_scene_upload(self.h, ctypes.byref(desc)))

    def render(self, cam, spp, max_depth, seed=1, precision=abi.RT_PREC_F32, tile_size=0, **kw):
        p = Context.params(spp, max_depth, seed, precision, **kw)
        out = np.zeros((cam.image_height, cam.image_width, 3),
                       dtype=np.float64 if precision == abi.RT_PREC_F64 else np.float32)
        self._check(self.lib.rt_multi_render(self.h, ctypes.byref(cam), ctypes.byref(p), tile_size, out.ctypes.data))
        return out

    def stats(self, rank):
        c = abi.rt_counters()
        self._check(self.lib.rt_multi_stats(self.h, rank, ctypes.byref(c)))
        return c


def multi_plan(w, h, ndev, rank, tile_size=0):
    """rt_multi_plan: the tiles rank `rank` renders (host only)."""
    L = abi.load()
    n = L.rt_multi_plan(w, h, ndev, tile_size, rank, None, 0)
    if n < 0:
        raise ValueError("invalid plan arguments")
    arr = (abi.rt_tile * max(1, n))()
    L.rt_multi_plan(w, h, ndev, tile_size, rank, arr, n)
    return [(t.x0, t.y0, t.width, t.height) for t in arr[:n]]
