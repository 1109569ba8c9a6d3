"""Dev tool: does PyTorch still see the GPU when librt_hip initialised HIP first? (r05v3 / r05h1: a
`-m gpu` test selection failed with "No HIP GPUs are available" in torch after rt_amd.Context.)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))
mode = sys.argv[1] if len(sys.argv) > 1 else "lib-first"
import torch  # noqa: E402

if mode != "lib-first-nocount":
    print("import: device_count", torch.cuda.device_count(), "initialized", torch.cuda.is_initialized(), flush=True)
if mode == "torch-first":
    torch.zeros(1, device="cuda")
    print("torch initialised first", flush=True)
import rt_amd  # noqa: E402

ctx = rt_amd.Context(0)
print("context created; device_count", torch.cuda.device_count(), flush=True)
maps = sorted(set(l.split()[-1] for l in open("/proc/self/maps") if "amdhip" in l or "hsa-runtime" in l))
print("runtimes", maps, flush=True)
try:
    x = torch.zeros(4, device="cuda")
    print("torch tensor ok", x.device, flush=True)
except Exception as e:  # noqa: BLE001
    print("torch failed:", type(e).__name__, e, flush=True)
ctx.close()
