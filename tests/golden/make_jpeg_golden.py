"""Generates the JPEG fixtures of tests/test_jpeg.py (run in the container that has /root/reference).

Inputs: the reference's earthmap.jpg (tests/golden/assets/) and small JPEGs written here with Pillow
in the layouts the decoder supports (4:4:4, 4:2:2, 4:2:0, 4:4:0, grayscale, restart intervals, odd
sizes) plus a progressive one it must refuse. Expected outputs: md5 of the 8-bit RGB pixels and of
the picture-texture bytes (float_to_byte(stbi_loadf)), as the reference's own decoder returns them:
its vendored stb_image.h compiled where it lies (oracle/Makefile `ref` -> oracle/_ref/stb_decode).

    make -C oracle ref && python tests/golden/make_jpeg_golden.py
"""
import hashlib
import json
import os
import subprocess

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
STB = os.path.join(REPO, "oracle", "_ref", "stb_decode")


def synthetic(w, h, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    img = np.stack([128 + 100 * np.sin(x / 5.0 + seed), 128 + 90 * np.cos(y / 7.0), (x * 3 + y * 5) % 256], -1)
    img += rng.normal(0, 12, img.shape)
    return Image.fromarray(np.clip(img, 0, 255).astype(np.uint8))


def cases():
    yield "earthmap.jpg", os.path.join(HERE, "assets", "earthmap.jpg"), None
    specs = [("s444", dict(subsampling=0), (64, 40)), ("s422", dict(subsampling=1), (61, 37)),
             ("s420", dict(subsampling=2), (67, 45)), ("s420_tiny", dict(subsampling=2), (9, 7)),
             ("restart", dict(subsampling=2, restart_marker_blocks=3), (64, 48)),
             ("gray", dict(), (50, 33)), ("q100", dict(subsampling=0, quality=100), (40, 40)),
             ("progressive", dict(progressive=True), (32, 32))]
    for name, kw, (w, h) in specs:
        im = synthetic(w, h, len(name))
        if name == "gray":
            im = im.convert("L")
        path = os.path.join(HERE, "jpeg", name + ".jpg")
        im.save(path, "JPEG", quality=kw.pop("quality", 85), **kw)
        yield name + ".jpg", path, kw


def main():
    out = {}
    for name, path, _ in cases():
        r = subprocess.run([STB, path], capture_output=True, text=True)
        if r.returncode != 0:
            out[name] = {"decodes": False}
            continue
        lines = r.stdout.split("\n")
        w, h = map(int, lines[0].split())
        out[name] = {"decodes": True, "width": w, "height": h,
                     "rgb_md5": hashlib.md5(bytes.fromhex(lines[1])).hexdigest(),
                     "texture_md5": hashlib.md5(bytes.fromhex(lines[2])).hexdigest()}
    out["_generator"] = "tests/golden/make_jpeg_golden.py: stb_image v2.30 from the reference (oracle/_ref/stb_decode)"
    with open(os.path.join(HERE, "jpeg_golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
