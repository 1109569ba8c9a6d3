"""Dev tool: where the wide-BVH persistent kernel's time goes (needs `make sections`). Renders a
bench config with the section-clock build and prints, per segment: node-loop and primitive-test
wave iterations with the lanes active in them, shade calls, and the trace / shade clock split.
    python3 scripts/dev_wide_stats.py c3 [f32|f64]"""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO + '/cpu-ray-tracing-implementation_amd/python')
sys.path.insert(0, REPO)
import rt_amd
from rt_amd import abi, plugin
import bench
abi.lib_path = lambda: os.environ.get('RT_HIP_LIB') or os.path.join(abi.BUILD_DIR, 'librt_hip_sections.so')
cfg = sys.argv[1] if len(sys.argv) > 1 else 'c3'
prec = abi.RT_PREC_F64 if (len(sys.argv) > 2 and sys.argv[2] == 'f64') else abi.RT_PREC_F32
name, w, aspect, spp, depth = bench.CONFIGS[cfg]
if name == 'sponza':
    bench.sponza_asset()
cs = plugin.ConfigScene(name, w, aspect)
ctx = rt_amd.Context(0)
ctx.upload(cs.desc)
lib = abi.load()
buf = (ctypes.c_ulonglong * 10)()
ctx.render(cs.cam, spp, depth, seed=1, precision=prec)
lib.rt_dev_wide_stats(buf)
ctx.reset_counters()
ctx.render(cs.cam, spp, depth, seed=1, precision=prec)
lib.rt_dev_wide_stats(buf)
segs = ctx.stats().segments
ni, nl, pi, pl, si, sl, ct, csh, fi, fl = list(buf)
print(f"{cfg} {name} {w}px {spp}spp d{depth} prec={prec}: segments {segs}")
print(f"  (flat / linear kernels: node loop = trace calls)")
print(f"  node loop: {ni / segs * 64:.2f} wave-iter x64 per segment, lanes/iter {nl / max(ni, 1):.1f} "
      f"(lane visits/segment {nl / segs:.2f})")
print(f"  prim tests: {pi / segs * 64:.2f} wave-iter x64 per segment, lanes/iter {pl / max(pi, 1):.1f} "
      f"(lane tests/segment {pl / segs:.2f})")
print(f"  shade: {si / segs * 64:.2f} wave-calls x64 per segment, lanes/call {sl / max(si, 1):.1f}")
print(f"  finished samples: {fi / segs * 64:.2f} wave-events x64 per segment, lanes/event {fl / max(fi, 1):.1f}")
print(f"  clocks: trace {ct / (ct + csh):.3f} shade {csh / (ct + csh):.3f}; wave-cycles per segment x64: "
      f"trace {ct / segs * 64:.0f} shade {csh / segs * 64:.0f}")
