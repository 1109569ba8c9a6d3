"""Generates the PNG and Radiance HDR fixtures of tests/test_png_hdr.py (run in the container that has
/root/reference).

Inputs: small files written here byte by byte -- PNG in every colour type and bit depth the format has
(gray 1/2/4/8/16, RGB 8/16, palette 1/2/4/8 with tRNS, gray+alpha and RGBA 8/16), each scanline filter and
a mixed-filter file, Adam7 interlacing at odd sizes, zlib streams with stored, fixed-Huffman and dynamic
blocks and IDAT split across chunks; HDR with new-style run-length scanlines (runs and dumps), flat pixels
(width < 8), zero exponents, an "#?RGBE" header with extra lines, and a file whose first scanline lacks
the RLE marker (stb's flat fallback). Expected outputs: md5 of the 8-bit RGB stbi_load returns (PNG) and
of the picture-texture bytes (float_to_byte(stbi_loadf)), as the reference's own decoder returns them:
its vendored stb_image.h compiled where it lies (oracle/Makefile `ref` -> oracle/_ref/stb_decode).

    make -C oracle ref && python tests/golden/make_image_golden.py
"""
import hashlib
import json
import os
import struct
import subprocess
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
STB = os.path.join(REPO, "oracle", "_ref", "stb_decode")
OUT = os.path.join(HERE, "images")


def chunk(t, data):
    return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xFFFFFFFF)


def paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def filter_rows(rows, bpp, filt):
    """rows: list of bytes (raw scanlines of one pass); filt: an int or a list of ints per row."""
    out = bytearray()
    prev = bytes(len(rows[0])) if rows else b""
    for y, row in enumerate(rows):
        f = filt[y % len(filt)] if isinstance(filt, list) else filt
        out.append(f)
        for i, x in enumerate(row):
            a = row[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            pred = [0, a, b, (a + b) >> 1, paeth(a, b, c)][f]
            out.append((x - pred) & 255)
        prev = row
    return bytes(out)


def pack_row(vals, depth):
    if depth == 8:
        return bytes(int(v) for v in vals)
    if depth == 16:
        return b"".join(struct.pack(">H", int(v)) for v in vals)
    out, acc, n = bytearray(), 0, 0
    for v in vals:
        acc = (acc << depth) | int(v)
        n += depth
        if n == 8:
            out.append(acc)
            acc, n = 0, 0
    if n:
        out.append(acc << (8 - n))
    return bytes(out)


def write_png(path, px, ctype, depth, filt=0, interlace=False, palette=None, trns=None, level=9, strategy=None,
              split=0):
    h, w, ch = px.shape
    bpp = max(1, (ch * depth) // 8)

    def scan(sub):
        return [pack_row(sub[y].reshape(-1), depth) for y in range(sub.shape[0])]
    if not interlace:
        raw = filter_rows(scan(px), bpp, filt)
    else:
        raw = b""
        for x0, y0, dx, dy in [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2),
                               (0, 1, 1, 2)]:
            sub = px[y0::dy, x0::dx]
            if sub.shape[0] and sub.shape[1]:
                raw += filter_rows(scan(sub), bpp, filt)
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 9, strategy if strategy is not None else zlib.Z_DEFAULT_STRATEGY)
    z = co.compress(raw) + co.flush()
    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, int(interlace)))
    if palette is not None:
        data += chunk(b"PLTE", bytes(palette))
    if trns is not None:
        data += chunk(b"tRNS", bytes(trns))
    if split:
        for i in range(0, len(z), split):
            data += chunk(b"IDAT", z[i:i + split])
    else:
        data += chunk(b"IDAT", z)
    data += chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(data)


def rgbe(rgb):
    """float RGB (h, w, 3) -> RGBE bytes (h, w, 4), as Radiance writes them (frexp of the max)."""
    m = rgb.max(-1)
    out = np.zeros(rgb.shape[:2] + (4,), np.uint8)
    nz = m > 1e-32
    mant, exp = np.frexp(m[nz])
    scale = mant * 256.0 / m[nz]
    out[nz, :3] = np.clip(rgb[nz] * scale[:, None], 0, 255).astype(np.uint8)
    out[nz, 3] = (exp + 128).astype(np.uint8)
    return out


def rle_component(vals):
    out, i, n = bytearray(), 0, len(vals)
    while i < n:
        j = i
        while j < n and j - i < 127 and vals[j] == vals[i]:
            j += 1
        if j - i >= 3:
            out += bytes([128 + (j - i), vals[i]])
            i = j
            continue
        j = i
        while j < n and j - i < 128 and not (j + 2 < n and vals[j] == vals[j + 1] == vals[j + 2]):
            j += 1
        out += bytes([j - i]) + bytes(vals[i:j])
        i = j
    return bytes(out)


def write_hdr(path, q, header=b"#?RADIANCE\n", extra=b"", rle=True, first_flat=False):
    h, w, _ = q.shape
    data = header + extra + b"FORMAT=32-bit_rle_rgbe\n\n" + f"-Y {h} +X {w}\n".encode()
    for y in range(h):
        if rle and not first_flat:
            data += bytes([2, 2, w >> 8, w & 255])
            for k in range(4):
                data += rle_component(list(q[y, :, k]))
        else:
            data += q[y].tobytes()
    with open(path, "wb") as f:
        f.write(data)


def cases():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(11)

    def img(h, w, ch, maxv, smooth=True):
        y, x = np.mgrid[0:h, 0:w]
        base = np.stack([(x * 7 + y * 3 + 31 * k) % (maxv + 1) for k in range(ch)], -1)
        noise = rng.integers(0, maxv + 1, (h, w, ch))
        return np.where(rng.random((h, w, ch)) < (0.2 if smooth else 0.8), noise, base).astype(np.int64)
    specs = []
    for f, name in enumerate(["none", "sub", "up", "avg", "paeth"]):
        specs.append((f"rgb8_{name}.png", img(13, 17, 3, 255), 2, 8, dict(filt=f)))
    specs += [
        ("rgb8_mixed.png", img(21, 19, 3, 255), 2, 8, dict(filt=[0, 1, 2, 3, 4, 4, 2])),
        ("rgba8.png", img(12, 15, 4, 255), 6, 8, dict(filt=[4, 1])),
        ("gray8.png", img(9, 23, 1, 255), 0, 8, dict(filt=[2, 3])),
        ("graya8.png", img(10, 11, 2, 255), 4, 8, dict(filt=[1, 4])),
        ("gray16.png", img(7, 9, 1, 65535), 0, 16, dict(filt=[4, 3])),
        ("rgb16.png", img(8, 10, 3, 65535), 2, 16, dict(filt=[1, 2, 4])),
        ("rgba16.png", img(6, 7, 4, 65535), 6, 16, dict(filt=[3])),
        ("graya16.png", img(5, 9, 2, 65535), 4, 16, dict(filt=[2])),
        ("gray1.png", img(11, 21, 1, 1), 0, 1, dict(filt=[0, 1, 4])),
        ("gray2.png", img(9, 13, 1, 3), 0, 2, dict(filt=[2, 4])),
        ("gray4.png", img(10, 7, 1, 15), 0, 4, dict(filt=[3, 1])),
        ("pal1.png", img(9, 19, 1, 1), 3, 1, dict(filt=[0, 4])),
        ("pal2.png", img(8, 11, 1, 3), 3, 2, dict(filt=[1])),
        ("pal4.png", img(12, 9, 1, 15), 3, 4, dict(filt=[2, 3], trns=list(range(0, 240, 16)))),
        ("pal8.png", img(14, 16, 1, 255), 3, 8, dict(filt=[4])),
        ("rgb8_adam7.png", img(13, 11, 3, 255), 2, 8, dict(filt=[4, 1, 2], interlace=True)),
        ("gray2_adam7.png", img(9, 10, 1, 3), 0, 2, dict(filt=[3], interlace=True)),
        ("pal4_adam7.png", img(11, 5, 1, 15), 3, 4, dict(filt=[1, 4], interlace=True)),
        ("rgba16_adam7.png", img(7, 9, 4, 65535), 6, 16, dict(filt=[2], interlace=True)),
        ("tiny_adam7.png", img(1, 1, 3, 255), 2, 8, dict(interlace=True)),
        ("stored.png", img(16, 20, 3, 255, smooth=False), 2, 8, dict(filt=[1], level=0)),
        ("fixed.png", img(16, 20, 3, 255), 2, 8, dict(filt=[2], strategy=getattr(zlib, "Z_FIXED", 4))),
        ("split_idat.png", img(30, 25, 3, 255), 2, 8, dict(filt=[4], split=37)),
    ]
    for name, px, ctype, depth, kw in specs:
        pal = None
        if ctype == 3:
            pal = [int(v) for v in rng.integers(0, 256, 3 << depth)]
        path = os.path.join(OUT, name)
        write_png(path, px, ctype, depth, palette=pal, **kw)
        yield name, path
    # Radiance HDR
    y, x = np.mgrid[0:6, 0:37]
    rgb = np.stack([0.001 + x / 9.0, 0.5 + 0.0 * x, np.exp((y - 3.0) * 1.7)], -1).astype(np.float64)
    rgb[2, 5:9] = 0.0  # zero exponents
    q = rgbe(rgb)
    q[4, 10:30] = q[4, 10]  # long runs
    for name, kw, qq in [("rle.hdr", {}, q), ("flat_narrow.hdr", dict(rle=False), q[:, :5].copy()),
                         ("rgbe_header.hdr", dict(header=b"#?RGBE\n", extra=b"# made by make_image_golden\nEXPOSURE=1.0\n"), q),
                         ("flat_wide.hdr", dict(first_flat=True), q)]:
        path = os.path.join(OUT, name)
        write_hdr(path, qq, **kw)
        yield name, path


def main():
    out = {}
    for name, path in cases():
        r = subprocess.run([STB, path], capture_output=True, text=True)
        if r.returncode != 0:
            out[name] = {"decodes": False}
            continue
        lines = r.stdout.split("\n")
        w, h = map(int, lines[0].split())
        out[name] = {"decodes": True, "width": w, "height": h,
                     "rgb_md5": hashlib.md5(bytes.fromhex(lines[1])).hexdigest(),
                     "texture_md5": hashlib.md5(bytes.fromhex(lines[2])).hexdigest()}
    out["_generator"] = "tests/golden/make_image_golden.py: stb_image v2.30 from the reference (oracle/_ref/stb_decode)"
    with open(os.path.join(HERE, "image_golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({k: v.get("decodes") for k, v in out.items() if not k.startswith("_")}))


if __name__ == "__main__":
    main()
