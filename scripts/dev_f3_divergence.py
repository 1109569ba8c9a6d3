"""Dev tool: where do the fp32 device paths of a config scene leave the fp64 ones?

  python scripts/dev_f3_divergence.py [SCENE WIDTH SPP DEPTH]        (default: perlin_texture_ball 100 64 5)

Renders the scene in both precisions, takes the pixels that differ most, finds their divergent samples
(one-sample renders with first_sample = s), and -- with `make trace` (build/librt_hip_trace.so) -- prints
the first such sample's segment trace in both precisions (a child process: the trace library is another
librt_hip)."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO + '/cpu-ray-tracing-implementation_amd/python')
import rt_amd  # noqa: E402
from rt_amd import abi, plugin  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != '--trace' else 'perlin_texture_ball'
w = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[1] != '--trace' else 100
spp = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[1] != '--trace' else 64
depth = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[1] != '--trace' else 5
F32, F64 = abi.RT_PREC_F32, abi.RT_PREC_F64

if sys.argv[1:2] == ['--trace']:  # child: one sample's trace in both precisions
    _, _, name, w, x, y, s, depth = sys.argv
    abi.lib_path = lambda: os.path.join(abi.BUILD_DIR, 'librt_hip_trace.so')
    cs = plugin.ConfigScene(name, int(w))
    ctx = rt_amd.Context(0)
    ctx.upload(cs.desc)
    for prec in (F32, F64):
        print(f'--- precision {"fp32" if prec == F32 else "fp64"}', flush=True)
        v = ctx.render(cs.cam, 1, int(depth), seed=7, precision=prec, tiles=[(int(x), int(y), 1, 1)],
                       first_sample=int(s))[0]
        print('value', v, flush=True)
    sys.exit(0)

cs = plugin.ConfigScene(name, w)
cam = cs.cam
ctx = rt_amd.Context(0)
ctx.upload(cs.desc)
i32 = ctx.render(cam, spp, depth, seed=7, precision=F32).astype(np.float64)
i64 = ctx.render(cam, spp, depth, seed=7, precision=F64)
d = np.abs(i32 - i64).max(-1)
rmse = np.sqrt(((i32 - i64) ** 2).reshape(-1, 3).mean(0))
print(f'{name} {cam.image_width}x{cam.image_height} {spp} spp depth {depth}: fp32 vs fp64 rmse {rmse}, '
      f'px > 1e-3: {int((d > 1e-3).sum())} of {d.size}', flush=True)
H, W = d.shape
first = None
print('  error histogram (px with max |d| above):', [(t, int((d > t).sum())) for t in (1e-6, 1e-5, 1e-4, 1e-3, 1e-2)], flush=True)
for i in np.argsort(d.ravel())[::-1][:int(os.environ.get('NTOP', '8'))]:
    y, x = divmod(int(i), W)
    bad = []
    for s in range(spp):
        a = ctx.render(cam, 1, depth, seed=7, precision=F32, tiles=[(x, y, 1, 1)], first_sample=s)[0].astype(np.float64)
        b = ctx.render(cam, 1, depth, seed=7, precision=F64, tiles=[(x, y, 1, 1)], first_sample=s)[0]
        if np.abs(a - b).max() > 1e-3:
            bad.append((s, a.round(4).tolist(), b.round(4).tolist()))
    print(f'  ({x},{y}) d={d[y, x]:.4g}: divergent samples {bad}', flush=True)
    if bad and first is None:
        first = (x, y, bad[0][0])
ctx.close()
if first and os.path.exists(os.path.join(abi.BUILD_DIR, 'librt_hip_trace.so')):
    x, y, s = first
    print(f'--- trace of ({x},{y}) sample {s}', flush=True)
    subprocess.run([sys.executable, os.path.abspath(__file__), '--trace', name, str(w), str(x), str(y), str(s),
                    str(depth)], check=True)
