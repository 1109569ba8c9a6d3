"""Framebuffer partitioning across ranks: 16x16 tiles dealt
round-robin, each rank renders its tiles packed in order, rank 0 gathers the
equal-size padded buffers and scatters them into the full framebuffer."""
import numpy as np

TILE = 16


def all_tiles(w, h, ts=TILE):
    return [(x, y, min(ts, w - x), min(ts, h - y)) for y in range(0, h, ts) for x in range(0, w, ts)]


def tiles_of(w, h, rank, world, ts=TILE):
    return all_tiles(w, h, ts)[rank::world]


def pixel_index(tiles, w):
    """Global pixel index (y*W + x) of every packed pixel of `tiles`, in packing order."""
    idx = [(np.mgrid[y0:y0 + th, x0:x0 + tw][0] * w + np.mgrid[y0:y0 + th, x0:x0 + tw][1]).reshape(-1)
           for (x0, y0, tw, th) in tiles]
    return np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)


def plan(w, h, world, ts=TILE):
    """Per-rank tiles, pixel counts and the padded per-rank buffer length."""
    tiles = [tiles_of(w, h, r, world, ts) for r in range(world)]
    counts = [sum(t[2] * t[3] for t in ts_) for ts_ in tiles]
    return tiles, counts, max(counts)
