"""Host output paths for a rendered framebuffer (H, W, 3), row 0 at the top (camera.h:170).

write_ppm reproduces the reference's P3 writer: header "P3\\nW H\\n255\\n" (camera.h:149-151), then
one "r g b" line per pixel with gamma 2.2 and int(255.999 * x) and no clamp (color.h:16-36), so
values above 1 give numbers above 255 exactly as the reference prints them. write_pfm / read_pfm
store the linear float framebuffer losslessly (Portable Float Map, little-endian, bottom row first).
"""
import numpy as np


def _gamma(x):
    with np.errstate(invalid="ignore"):
        return np.where(x > 0, np.power(np.where(x > 0, x, 1.0), 1 / 2.2), 0.0)  # color.h:16-20 (NaN -> 0)


def ppm_bytes(image):
    img = np.asarray(image, dtype=np.float64)
    h, w = img.shape[:2]
    v = np.trunc(255.999 * _gamma(img.reshape(-1, 3))).astype(np.int64)  # int(...) truncates toward 0
    lines = "\n".join(f"{r} {g} {b}" for r, g, b in v)
    return f"P3\n{w} {h}\n255\n{lines}\n".encode()


def write_ppm(image, path):
    with open(path, "wb") as f:
        f.write(ppm_bytes(image))


def write_pfm(image, path):
    img = np.asarray(image, dtype=np.float32)
    h, w = img.shape[:2]
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(np.ascontiguousarray(img[::-1].astype("<f4")).tobytes())


def read_pfm(path):
    with open(path, "rb") as f:
        kind = f.readline().strip()
        if kind not in (b"PF", b"Pf"):
            raise ValueError("not a PFM file")
        w, h = (int(x) for x in f.readline().split())
        scale = float(f.readline())
        ch = 3 if kind == b"PF" else 1
        data = np.frombuffer(f.read(), dtype="<f4" if scale < 0 else ">f4", count=w * h * ch)
    return data.reshape(h, w, ch)[::-1].astype(np.float32)
