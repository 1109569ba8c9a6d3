"""Dev tool: where k_step's time goes (needs `make sections`). Renders a config with the
section-clock build and prints cycles per lane-segment for trace / shade / state store."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO + '/cpu-ray-tracing-implementation_amd/python')
import rt_amd
from rt_amd import abi, plugin
abi.lib_path = lambda: os.path.join(abi.BUILD_DIR, 'librt_hip_sections.so')
name, w, spp, depth = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else ('cornell_box', 800, 64, 50)
K = int(os.environ.get('RT_K', '16'))  # section clocks live in k_step (wavefront schedule)
cs = plugin.ConfigScene(name, w, 1.5 if name == 'rtow' else 1.0)
ctx = rt_amd.Context(0)
ctx.upload(cs.desc)
lib = abi.load()
buf = (ctypes.c_ulonglong * 7)()
ctx.render(cs.cam, spp, depth, seed=1, segments_per_launch=K)
lib.rt_dev_section_clocks(buf)
ctx.reset_counters()
ctx.render(cs.cam, spp, depth, seed=1, segments_per_launch=K)
lib.rt_dev_section_clocks(buf)
segs = ctx.stats().segments
tr, sh, st, lanes, pops, nodes, prims = list(buf)
print(f"{name} {w}px {spp}spp d{depth}: segments {segs}, lane-launches {lanes}")
print(f"  cycles per segment: trace {tr / segs:.0f}  shade {sh / segs:.0f}  (store per lane-launch {st / lanes:.0f})")
print(f"  shares: trace {tr / (tr + sh):.3f} shade {sh / (tr + sh):.3f}")
if pops:
    print(f"  BVH per segment: pops {pops / segs:.2f}  node pops {nodes / segs:.2f}  primitive tests {prims / segs:.2f}")
