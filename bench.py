#!/usr/bin/env python3
"""Msamples/s of the MI355X wavefront path tracer on BASELINE.json's headline config.

Workload (BASELINE.json configs[1]): the reference's Cornell Box
(main.cc:198-225) at 800x800, 1024 spp, max depth 50, light importance sampling on.
One step = one full frame. The framebuffer is cut into 16x16 tiles dealt
round-robin to the ranks; each rank renders its tiles on its GPU and rank 0
gathers them (RCCL, torch.distributed "nccl") into the full linear framebuffer.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)
"""
import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rt_amd  # noqa: E402
from rt_amd import abi, buildinfo, plugin  # noqa: E402
from rt_amd.distributed import FrameSharding  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
SIMDS, CLOCK_GHZ = 1024, 2.4  # 256 CUs x 4 SIMDs; the 2.4 GHz peak engine clock (MI355X_MICROARCH.md)
CYCLE_PEAK_G = SIMDS * CLOCK_GHZ  # G SIMD-cycles/s: every SIMD issuing VALU work every cycle
# VALU roofline: SIMD cycles per launch = sum over the kernel's VALU instructions of the cycles
# each holds its SIMD, measured on this MI355X for single opcodes (tools/valu_rates.hip, 8 waves/SIMD, 8
# independent chains; kernel time x the measured shader clock: profiles/r04t_valu_rates.json, 79 opcodes) and
# rounded to the issue cost they show: 2 cycles per wave64 instruction for 32-bit add/sub/mul/fma, and/or/
# xor/not/bitop3, moves and right shifts (measured 2.2-2.4); 4 for every fp64 operation, 64-bit moves and
# shifts, conversions, min/max/med3 of any type, the three-operand integer ops (add3, lshl_add, lshl_or,
# or3, and_or, xad, perm, bfi, alignbit, mad/mul_u32_u24), 32-bit integer multiplies, left shifts,
# bit-field extracts, fp32 floor/fract/ldexp, v_fma_mix and v_cndmask with an SGPR mask (4.1-4.3); 4.7 for
# compares into an SGPR mask (VOPC, any width); 5.0 for v_mad_u64_u32, 5.9 for v_readfirstlane, 8 for fp32
# transcendentals (8.1) and 16 for fp64 ones (16.2). Opcodes the table measured take their rounded
# measurement; the others the rules in opcode_cycles.
VALU_RATES = os.path.join(REPO, "profiles", "r04t_valu_rates.json")
VALU_PMC_CLASSES = {  # SQ_INSTS_VALU_* class counters -> the static-mix class they count
    "f64_addmulfma": ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64"),
    "f64_trans": ("SQ_INSTS_VALU_TRANS_F64",),
    "f32_trans": ("SQ_INSTS_VALU_TRANS_F32",),
    "cvt": ("SQ_INSTS_VALU_CVT",),
    "int64": ("SQ_INSTS_VALU_INT64",),
    # 32-bit integer instructions (round 5: counted, so that under half of the instructions -- moves, selects,
    # compares, fp32 and the fp64 opcodes no counter singles out -- are priced by the static mix)
    "int32_other": ("SQ_INSTS_VALU_INT32",),
}


_MEASURED = None


def _round_cost(c):
    """A measured cycles-per-instruction figure (event time, so a few % over the issue cost) -> the cost."""
    for lo, cost in ((14.0, 16.0), (7.0, 8.0), (5.5, 5.9), (4.9, 5.0), (4.5, 4.7), (3.0, 4.0)):
        if c >= lo:
            return cost
    return 2.0


def opcode_cycles(op):
    """Issue cycles of one wave64 VALU opcode on gfx950 (the table above)."""
    import re
    global _MEASURED
    if _MEASURED is None:
        _MEASURED = {}
        if os.path.exists(VALU_RATES):
            with open(VALU_RATES) as f:
                for name, v in json.load(f)["per_wave_instr"].items():
                    if name.startswith("v_cndmask"):  # the table's v_cndmask rows time mask set-up too
                        continue
                    _MEASURED[name] = _round_cost(v["cycles_event"])
    base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    if base in _MEASURED:
        return _MEASURED[base]
    if re.match(r"v_(rcp|rsq|sqrt|exp|log|sin|cos)_f64", op):
        return 16.0
    if re.match(r"v_(rcp|rsq|sqrt|exp|log|sin|cos|rcp_iflag)_f32", op):
        return 8.0
    if op.startswith("v_cmp"):
        return 4.7
    if op.startswith(("v_mad_u64_u32", "v_mad_i64_i32")):
        return 5.0
    if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
        return 5.9
    if ("f64" in op or "_b64" in op or "_u64" in op or "_i64" in op or op.startswith(("v_cvt", "v_bfe", "v_pk_"))
            or re.match(r"v_mul_(lo|hi)_", op) or re.match(r"v_(min|max|med3|min3|max3)_", op)
            or re.match(r"v_(add3|lshl_add|lshl_or|or3|and_or|xad|perm|bfi|alignbit|mad_u32_u24|mad_i32_i24|"
                        r"mul_u32_u24|mul_i32_i24|mul_hi_u32_u24|ldexp|fract|floor|ceil|trunc|rndne|fma_mix|"
                        r"mad_mix|lshlrev_b32|sad)", op)
            or op.startswith("v_cndmask_b32_e64")):
        return 4.0
    return 2.0


def issue_cycles(counters, mix):
    """SIMD cycles per launch: the classes the SQ_INSTS_VALU_* counters count, each at the mean cost of its
    opcodes in the kernel's static mix (scripts/valu_static_mix.py), and the remaining VALU instructions at
    the mean cost of the remaining opcodes -- fp64 compares, min/max and the like included. Returns
    (cycles, {class: (instructions, cycles per instruction)})."""
    import sys as _s
    _s.path.insert(0, os.path.join(REPO, "scripts"))
    from valu_static_mix import classify
    ops = mix["opcodes"]
    by_class = {}
    for op, n in ops.items():
        by_class.setdefault(classify(op), []).append((op, n))

    def mean_cost(items, default):
        tot = sum(n for _, n in items)
        return sum(opcode_cycles(op) * n for op, n in items) / tot if tot else default
    parts, counted = {}, 0.0
    for cl, names in VALU_PMC_CLASSES.items():
        if all(k in counters for k in names):
            n = sum(counters[k] for k in names)
            parts[cl] = (n, mean_cost(by_class.get(cl, []), opcode_cycles({"f64_addmulfma": "v_add_f64",
                                                                           "f64_trans": "v_rcp_f64",
                                                                           "f32_trans": "v_rcp_f32",
                                                                           "cvt": "v_cvt_f32_f64",
                                                                           "int64": "v_lshl_add_u64",
                                                                           "int32_other": "v_add_u32"}[cl])))
            counted += n
    rest_items = [(op, n) for cl, items in by_class.items() if cl not in parts for op, n in items]
    parts["rest"] = (max(0.0, counters["SQ_INSTS_VALU"] - counted), mean_cost(rest_items, 2.0))
    return sum(n * c for n, c in parts.values()), parts


# SURVEY.md §8(d) algorithmic bytes: per sample (generate + finalise) and per segment
B_GEN, B_ACC, B_EXT, B_SHADE = 64, 36, 44, 152

CONFIGS = {
    # name: (scene, width, aspect, spp, depth)
    "c1": ("cornell_box", 400, 1.0, 64, 8),
    "c2": ("cornell_box", 800, 1.0, 1024, 50),
    "c3": ("rtow", 1200, 1.5, 512, 50),
    "c4": ("sponza", 1920, 16.0 / 9.0, 256, 5),
    "c5": ("cornell_box_with_volume", 3840, 16.0 / 9.0, 4096, 5),
    # SURVEY §8(f) rows (not BASELINE configs): main.cc's own sizes and spp, on the CAMX kernels
    "f1": ("skybox_and_fisheye", 600, 1.0, 500, 5),       # main.cc:174-183: fisheye camera, picture skybox
    "f2": ("skybox_and_motion_blur", 600, 1.0, 500, 5),   # main.cc:185-196: earthmap texture, moving sphere
    "f3": ("perlin_texture_ball", 600, 1.0, 500, 5),      # main.cc:402-437: perlin textures over 400 boxes
}


def sponza_asset():
    """C4's glTF: $RT_SPONZA_GLTF (the real Sponza, if supplied), else the synthetic stand-in
    (rt_amd.synth_gltf: 262,267 triangles, same camera and light) written to a temp directory."""
    path = os.environ.get("RT_SPONZA_GLTF")
    if path and os.path.exists(path):
        return path, "Sponza glTF " + path
    import tempfile
    from rt_amd import synth_gltf
    path = synth_gltf.write_sponza_standin(tempfile.mkdtemp(prefix="sponza_standin_"))
    os.environ["RT_SPONZA_GLTF"] = path
    return path, "synthetic Sponza stand-in (rt_amd.synth_gltf, 262,267 triangles; Sponza.bin is not shipped)"


def cpu_threads():
    """Threads for the CPU baseline: every CPU this process may use, capped by the box's CPU share
    (cgroup quota, or OMP_NUM_THREADS, which the GPU box sets to its share)."""
    info = buildinfo.host_cpu()
    n = info["affinity"]
    if info["cgroup_quota_cpus"]:
        n = min(n, max(1, int(info["cgroup_quota_cpus"])))
    if info["omp_num_threads"]:
        try:
            n = min(n, max(1, int(info["omp_num_threads"])))
        except ValueError:
            pass
    return n, info


def lit_tiles(fb, W, H, ts=16, seed=7):
    """16x16 tiles for C4's sample: the frame's tiles ordered brightest first (by the GPU frame just
    rendered), interleaved with a seeded random order, so the sample covers lit pixels and not only the
    dark rows a row sample of the stand-in picks (round-3 verdict: 2 near-black rows)."""
    img = fb.reshape(H, W, 3).double().cpu().numpy().mean(-1)
    tiles = [(x, y, min(ts, W - x), min(ts, H - y)) for y in range(0, H, ts) for x in range(0, W, ts)]
    lum = [float(img[y:y + h, x:x + w].mean()) for (x, y, w, h) in tiles]
    bright = sorted(range(len(tiles)), key=lambda i: -lum[i])
    rnd = np.random.default_rng(seed).permutation(len(tiles)).tolist()
    order, seen = [], set()
    for i, j in zip(bright, rnd):
        for k in (i, j):
            if k not in seen:
                seen.add(k)
                order.append(tiles[k])
    return order


def cpu_baseline(scene_name, width, aspect, spp, depth, seed, threads, target_msamples, budget_s=25.0, tiles=None):
    """The oracle (fp64 restatement of the reference loop, counter RNG) on host cores, over a sample of the
    frame: evenly spaced full rows, or (tiles) the first of the given tiles that fit the time budget.
    Returns (the bench line's cpu_baseline object, the sampled tiles, their fp64 pixels (packed))."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    cs = plugin.ConfigScene(scene_name, width, aspect)
    cam = cs.cam
    osc = oracle.from_desc(cs.desc)
    H, W = cam.image_height, cam.image_width
    t0 = time.perf_counter()
    if tiles is None:
        # evenly spaced full rows at the full spp and depth: about target_msamples of work, cut to what fits
        # in budget_s on this host (a middle row is timed first: the top rows of a frame can be cheap)
        nrows = max(1, min(H, int(target_msamples * 1e6 // (W * spp))))
        probe = H // 2
        first, segs = oracle.render(osc, cam, spp, depth, seed=seed, threads=threads, tiles=[(0, probe, W, 1)])
        t_unit = time.perf_counter() - t0
        nrows = max(1, min(nrows, int(budget_s / max(t_unit, 1e-6))))
        rows = sorted(set(int(round(x)) for x in np.linspace(0, H - 1, nrows)))
        k = min(range(len(rows)), key=lambda i: abs(rows[i] - probe))  # the timed row stands in for its neighbour
        rows[k] = probe
        rows = sorted(set(rows))
        order = [(0, probe, W, 1)] + [(0, y, W, 1) for y in rows if y != probe]
        what = f"{len(rows)} evenly spaced rows x {W} px"
        want = len(order)
    else:
        order = list(tiles)
        first, segs = oracle.render(osc, cam, spp, depth, seed=seed, threads=threads, tiles=order[:1])
        t_unit = time.perf_counter() - t0
        want = max(1, min(len(order), int(budget_s / max(t_unit, 1e-6))))
    print(f"cpu_baseline: first unit {t_unit:.2f} s, rendering up to {want}", file=sys.stderr, flush=True)
    done = [first]
    sample = [order[0]]
    batch_n = 16 if tiles is None else 8
    i = 1
    while i < want and (tiles is None or time.perf_counter() - t0 < budget_s):
        batch = order[i:min(want, i + batch_n)]
        img, sg = oracle.render(osc, cam, spp, depth, seed=seed, threads=threads, tiles=batch)
        segs += sg
        done.append(img)
        sample += batch
        i += len(batch)
        print(f"cpu_baseline: {len(sample)}/{want} units, {time.perf_counter() - t0:.1f} s", file=sys.stderr,
              flush=True)
    dt = time.perf_counter() - t0
    img = np.concatenate(done)
    npx = sum(t[2] * t[3] for t in sample)
    if tiles is not None:
        what = f"{len(sample)} 16x16 tiles (brightest first, interleaved with random ones; {npx} px)"
    n = npx * spp
    n_threads, info = threads, buildinfo.host_cpu()
    line = {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": n_threads, "kind": "port",
            "per_core": round(n / dt / 1e6 / n_threads, 4),
            "segments_per_sample": round(segs / n, 4),
            "msegments_per_s": round(segs / dt / 1e6, 3),
            "host": info,
            "sample": f"oracle (fp64 C++ restatement of camera.h:135-241, counter RNG, std::thread pool of "
                      f"{n_threads}) on {what} x {spp} spp, depth {depth}: {n / 1e6:.1f} Msamples "
                      f"({segs / 1e6:.1f} M segments) in {dt:.1f} s"}
    return line, sample, img


def parity_tiles(fb, W, tiles, ref, rel_tol=None):
    """The GPU framebuffer's pixels of `tiles` against the oracle's (same seed, same sample streams):
    SURVEY.md §8(c) link 3, at the full bench config. fp32: per-channel RMSE < 1e-4 (north_star). fp64
    (rel_tol): also the count of pixels differing by more than rel_tol relative (the -m gpu tests hold
    fp64 to 1e-9 in all but a few pixels). mean_radiance shows the compared pixels are not black, beside
    the whole GPU frame's (frame_mean_radiance: the C4 stand-in is a dim scene, its light quad high above
    the geometry)."""
    from rt_amd.tiling import pixel_index
    idx = torch.from_numpy(pixel_index(tiles, W)).to(fb.device)
    got = fb[idx].double().cpu().numpy()
    d = got - ref
    rmse = np.sqrt((d ** 2).reshape(-1, 3).mean(0))
    out = {"rmse": [float(f"{x:.3g}") for x in rmse], "max_abs": float(f"{np.abs(d).max():.3g}"),
           "tiles": len(tiles), "pixels": int(d.shape[0]), "tolerance": 1e-4,
           "mean_radiance": float(f"{ref.mean():.4g}"), "lit_pixels": int((ref.max(-1) > 1e-3).sum()),
           "frame_mean_radiance": float(f"{fb.double().mean().item():.4g}"),
           "pass": bool((rmse < 1e-4).all() and np.isfinite(got).all()),
           "against": "oracle fp64, same seed and counter-RNG streams"}
    if rel_tol is not None:
        bad = (np.abs(d) > rel_tol * np.maximum(1.0, np.abs(ref))).any(-1)
        out.update({"rel_tol": rel_tol, "pixels_over_rel_tol": int(bad.sum()),
                    "max_rel": float(f"{(np.abs(d) / np.maximum(1.0, np.abs(ref))).max():.3g}")})
    return out


def lit_parity(ctx, width, aspect, spp, depth, seed, threads, precisions, budget_s=20.0, ts=16, gpu_tiles=400):
    """C4's kernel and tree on lit pixels (round-4 verdict): `sponza_lit` is the C4 stand-in -- the same
    262,267 triangles, the same tree, the reference's light -- plus one unsampled diffuse_light quad under the
    stand-in's grid over the camera (scenes/config_scenes.cpp). Seeded random 16x16 tiles of the full
    1920x1080 frame at C4's own spp and depth, the oracle's first tiles that fit `budget_s`, against the GPU's
    same tiles in each precision. Runs after the timed region (it uploads another scene)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    cs = plugin.ConfigScene("sponza_lit", width, aspect)
    cam = cs.cam
    W, H = cam.image_width, cam.image_height
    tiles = [(x, y, min(ts, W - x), min(ts, H - y)) for y in range(0, H, ts) for x in range(0, W, ts)]
    order = [tiles[i] for i in np.random.default_rng(seed + 11).permutation(len(tiles))]
    osc = oracle.from_desc(cs.desc)
    t0 = time.perf_counter()
    done, sample = [], []
    while order and time.perf_counter() - t0 < budget_s:
        batch, order = order[:4], order[4:]
        img, _ = oracle.render(osc, cam, spp, depth, seed=seed, threads=threads, tiles=batch)
        done.append(img)
        sample += batch
    ref = np.concatenate(done)
    st, info, _ = abi.scene_check(cs.desc)
    # a tree takes the LDS-resident kernel only when all of it fits a block's 40 KiB (rt_kernels.hip
    # wide_lds_bytes; a node is >= 48 B there): C4's 59,888 nodes take the HBM kernel C4 times
    out = {"scene": "sponza_lit: the C4 stand-in + a second (unsampled) light under its grid over the camera",
           "triangles": info.triangles, "wide_nodes": info.wide_nodes, "tree_in_hbm": info.wide_nodes * 48 > 40 << 10,
           "oracle_s": round(time.perf_counter() - t0, 1)}
    ctx.upload(cs.desc)
    for prec in precisions:
        got = ctx.render(cam, spp, depth, seed=seed, precision=prec, tiles=sample).astype(np.float64)
        d = got - ref
        rmse = np.sqrt((d ** 2).reshape(-1, 3).mean(0))
        r = {"rmse": [float(f"{x:.3g}") for x in rmse], "max_abs": float(f"{np.abs(d).max():.3g}"),
             "tiles": len(sample), "pixels": int(d.shape[0]), "mean_radiance": float(f"{ref.mean():.4g}"),
             "lit_pixels": int((ref.max(-1) > 1e-3).sum()), "tolerance": 1e-4,
             "pass": bool((rmse < 1e-4).all() and np.isfinite(got).all())}
        if prec == abi.RT_PREC_F64:
            bad = (np.abs(d) > 1e-9 * np.maximum(1.0, np.abs(ref))).any(-1)
            r.update({"rel_tol": 1e-9, "pixels_over_rel_tol": int(bad.sum())})
        out["fp64" if prec == abi.RT_PREC_F64 else "fp32"] = r
    # a larger sample without the oracle: fp32 against the GPU's fp64, which follows the oracle to 1e-9 on the
    # tiles above, over the first gpu_tiles seeded tiles (round 6: the 24 oracle tiles read 9.2e-5 where 400 tiles
    # read 1.7e-4 -- the fp32 paths' rounding decides a few samples per tile near edges and plane crossings)
    if abi.RT_PREC_F32 in precisions and abi.RT_PREC_F64 in precisions:
        big = [tiles[i] for i in np.random.default_rng(seed + 11).permutation(len(tiles))][:gpu_tiles]
        a = ctx.render(cam, spp, depth, seed=seed, precision=abi.RT_PREC_F32, tiles=big).astype(np.float64)
        b = ctx.render(cam, spp, depth, seed=seed, precision=abi.RT_PREC_F64, tiles=big)
        d = (a - b).reshape(-1, 3)
        rmse = np.sqrt((d ** 2).mean(0))
        out["fp32_vs_fp64_gpu"] = {"tiles": len(big), "pixels": int(d.shape[0]),
                                   "rmse": [float(f"{x:.3g}") for x in rmse],
                                   "pixels_over_1e-3": int((np.abs(d).max(-1) > 1e-3).sum()),
                                   "mean_radiance": float(f"{b.mean():.4g}"), "tolerance": 1e-4,
                                   "pass": bool((rmse < 1e-4).all())}
    return out


class Hip:
    """The few HIP runtime calls bench.py's copy stream needs, through ctypes, bound to the HIP runtime this
    process already runs on (torch's bundled libamdhip64.so.7, which librt_hip shares): found in /proc/self/maps
    and opened with RTLD_NOLOAD, so a second runtime (/opt/rocm's, by an unversioned name) is never loaded and
    the stream and event handles torch hands over stay valid. Fails loudly if no runtime is loaded yet."""

    def __init__(self):
        import ctypes
        self.ct = ctypes
        path = None
        with open("/proc/self/maps") as fh:
            for line in fh:
                f = line.split()
                if len(f) >= 6 and os.path.basename(f[5]).startswith("libamdhip64.so"):
                    path = f[5]
                    break
        if path is None:
            raise RuntimeError("bench.py: no HIP runtime is loaded in this process (torch is imported and the "
                               "GPU touched before Hip())")
        self.lib = ctypes.CDLL(path, mode=os.RTLD_NOLOAD | os.RTLD_NOW)
        for name, args in (("hipEventCreateWithFlags", [ctypes.c_void_p, ctypes.c_uint]),
                           ("hipEventRecord", [ctypes.c_void_p, ctypes.c_void_p]),
                           ("hipStreamWaitEvent", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]),
                           ("hipMemcpyAsync", [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                               ctypes.c_void_p])):
            getattr(self.lib, name).argtypes = args
            getattr(self.lib, name).restype = ctypes.c_int

    def _ok(self, e, what):
        if e != 0:
            raise RuntimeError(f"{what} failed: hip error {e}")

    def event(self):
        ev = self.ct.c_void_p()
        self._ok(self.lib.hipEventCreateWithFlags(self.ct.byref(ev), 2), "hipEventCreateWithFlags")  # no timing
        return ev

    def record(self, ev, stream):
        self._ok(self.lib.hipEventRecord(ev, self.ct.c_void_p(stream)), "hipEventRecord")

    def wait(self, stream, ev):
        self._ok(self.lib.hipStreamWaitEvent(self.ct.c_void_p(stream), ev, 0), "hipStreamWaitEvent")

    def d2h(self, dst, src, nbytes, stream):
        self._ok(self.lib.hipMemcpyAsync(self.ct.c_void_p(dst), self.ct.c_void_p(src), nbytes, 2,
                                         self.ct.c_void_p(stream)), "hipMemcpyAsync")


def measured_pmc(workload):
    """Per-launch PMC figures of the dominant kernel for this exact workload and build (profiles/*_pmc.json,
    written by scripts/pmc_summary.py from separate rocprofv3 --pmc passes; the last in name order wins),
    or None when no pass was collected on this build."""
    found = None
    sha = buildinfo.src_sha()
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc.json"))):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("workload") == workload and d.get("src_sha") == sha:
            found = (os.path.basename(f), d)
    return found


def workload_key(scene_name, W, H, spp, depth, args, precision=None):
    return (f"{scene_name} {W}x{H} {spp}spp depth {depth} {precision or args.precision} pool={args.pool} "
            f"chunk={args.chunk} "
            f"K={args.segments_per_launch} world={args.gpus}" + (" ordered" if args.traversal == "ordered" else ""))


def roofline(key, st, segs, my_samples, elapsed, kern, fp64):
    """The dominant kernel's roofline: VALU issue per launch from the PMC summary of this
    build and workload (profiles/*_pmc.json) over the launch time measured live with HIP events."""
    iters, step_ms = st.iterations, st.step_ms
    if iters <= 0 or step_ms <= 0:
        return None
    alg_bytes = (B_GEN + B_ACC) * my_samples + (B_EXT + B_SHADE) * segs
    avg_s = step_ms / 1e3 / iters
    mp = measured_pmc(key)
    roof = {"bound": "valu", "kernel": kern, "unit": "G SIMD-cycles/s", "peak": CYCLE_PEAK_G,
            "achieved": None, "frac": None, "traffic": None,
            "avg_launch_us": round(avg_s * 1e6, 2), "launches": iters,
            "kernel_share_of_wall": round(step_ms / 1e3 / elapsed, 4),
            "wavefront_equiv": {"alg_bytes_per_launch": int(alg_bytes / iters),
                                "GBps": round(alg_bytes / (step_ms / 1e3) / 1e9, 1),
                                "note": "SURVEY §8(d) bytes a classic SoA wavefront would move for "
                                        "this work; not HBM traffic"}}
    if not mp:
        return roof
    d = mp[1]
    c = dict(d.get("counters", {}))
    c["SQ_INSTS_VALU"] = d["valu_per_launch"]
    mix = None
    if d.get("valu_mix"):
        with open(os.path.join(REPO, "profiles", d["valu_mix"])) as fh:
            mix = json.load(fh)
    roof.update({"valu_per_launch": d["valu_per_launch"], "pmc_source": "profiles/" + mp[0],
                 "lane_valu_per_segment": round(d["valu_per_launch"] * 64 / (segs / iters), 1),
                 "valu_lane_util": d.get("valu_lane_util"), "wait_frac": d.get("wait_frac")})
    if mix is None:  # no static mix of this build: instructions at 2 cycles, the counted fp64 ones at 4
        n64 = sum(c.get(k, 0.0) for k in VALU_PMC_CLASSES["f64_addmulfma"] + VALU_PMC_CLASSES["f64_trans"])
        cycles, parts = 2.0 * (d["valu_per_launch"] - n64) + 4.0 * n64, None
    else:
        cycles, parts = issue_cycles(c, mix)
    ach = cycles / avg_s / 1e9
    gui = d.get("grbm_gui_active_per_launch")
    tr = d.get("trace_avg_ns")
    roof.update({"unit": "G SIMD-cycles/s", "peak": CYCLE_PEAK_G, "achieved": round(ach, 2),
                 "frac": round(ach / CYCLE_PEAK_G, 4), "valu_cycles_per_launch": cycles,
                 # the same cycles over the profiled run's kernel-trace duration (profiles/*_kernel_stats.csv):
                 # what the committed profile alone gives; frac = frac_profiled * trace_avg / live launch time
                 "frac_profiled": round(cycles / (tr * 1e-9) / 1e9 / CYCLE_PEAK_G, 4) if tr else None,
                 "trace_avg_us": round(tr / 1e3, 2) if tr else None,
                 "profiled_clock_ghz": d.get("profiled_clock_ghz"),
                 # the live launch at the profiled run's clock: the two runs' clocks differ from box to box
                 "live_clock_ghz_equiv": (round(d["profiled_clock_ghz"] * tr * 1e-9 / avg_s, 3)
                                          if tr and d.get("profiled_clock_ghz") else None),
                 # the same cycles against the cycles the GPU was active during the profiled launches
                 # (GRBM_GUI_ACTIVE / 8 XCDs): independent of the clock
                 "frac_at_measured_clock": round(cycles / (SIMDS * gui / 8), 4) if gui else None,
                 "cycles_by_class": ({k: {"instr": round(n), "cycles_per_instr": round(cc, 3)} for k, (n, cc) in
                                      parts.items()} if parts else None),
                 "valu_mix": ("profiles/" + d["valu_mix"]) if d.get("valu_mix") else None,
                 "peak_basis": "1024 SIMDs x 2.4 GHz; SIMD cycles per VALU opcode measured (tools/valu_rates.hip, "
                               "profiles/r04c_valu_rates.json): 2 for 32-bit add/mul/fma/logic, 4 for fp64 and "
                               "64-bit ops, conversions, SGPR-mask selects, 4.6 compares, 8 / 16 fp32 / fp64 "
                               "transcendentals; per-class counts from SQ_INSTS_VALU_* counters, the rest at "
                               "the kernel's static opcode mix"})
    if d.get("tcp_accesses_per_launch"):
        # the L1 / texture-address path: the TA units process about one cache access per clock per CU, and
        # a kernel whose node and primitive fetches keep them busy every cycle (C4's tree in HBM) is bound
        # there, whatever its VALU fraction: then that is the roofline reported
        acc = d["tcp_accesses_per_launch"]
        ta = {"achieved": round(acc / avg_s / 1e9, 2), "peak": round(256 * CLOCK_GHZ, 1),
              "unit": "G L1 accesses/s (TCP_TOTAL_CACHE_ACCESSES)", "frac": round(acc / avg_s / 1e9 / (256 * CLOCK_GHZ), 4),
              "ta_busy_frac": d.get("ta_busy_frac"), "accesses_per_launch": acc}
        roof["l1"] = ta
        if ta["frac"] > roof["frac"]:
            valu = {k: roof[k] for k in ("unit", "achieved", "peak", "frac", "valu_cycles_per_launch",
                                         "frac_at_measured_clock", "cycles_by_class", "valu_mix", "peak_basis")}
            roof.update({"bound": "l1_ta", "unit": ta["unit"], "achieved": ta["achieved"], "peak": ta["peak"],
                         "frac": ta["frac"], "valu": valu,
                         "peak_basis": "256 CUs x 2.4 GHz x 1 L1 (TCP) access per clock: TA busy "
                                       f"{d.get('ta_busy_frac')} of the active cycles (TA_TA_BUSY / GRBM_GUI_ACTIVE)"})
    if roof["valu_lane_util"] is not None:  # issued lanes that do work: idle lanes of a divergent wave do not
        vf = roof["frac"] if roof["bound"] == "valu" else roof["valu"]["frac"]
        roof["useful_frac"] = round(vf * roof["valu_lane_util"], 4)
    if d.get("hbm_bytes_per_launch") is not None:
        tb = d["hbm_bytes_per_launch"]
        roof["traffic"] = int(tb)
        roof["hbm"] = {"achieved_GBps": round(tb / avg_s / 1e9, 2), "peak_GBps": HBM_PEAK_GBS,
                       "frac": round(tb / avg_s / 1e9 / HBM_PEAK_GBS, 5)}
    assert roof["frac"] <= 1.0, roof
    return roof


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)  # 10 frames: 0.25 s on one GPU, 36 ms over 8
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    # the headline computes in fp64, the reference's precision (vec3.h:7); the fp32 production path, which
    # meets north_star's per-channel RMSE < 1e-4, is timed after it as the "alt" line
    ap.add_argument("--precision", default="f64", choices=["f32", "f64"])
    ap.add_argument("--pool", type=int, default=0, help="path slots / persistent lanes (0 = library default)")
    ap.add_argument("--chunk", type=int, default=0, help="samples per work item (0 = library default)")
    ap.add_argument("--segments-per-launch", type=int, default=0,
                    help="0: persistent schedule (one k_persist launch per frame); K > 0: "
                         "wavefront k_step launches of K segments per path slot")
    ap.add_argument("--traversal", default="auto", choices=["auto", "ordered"],
                    help="ordered: the reference-ordered linear program / BVH also in fp32 (no flat program)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--kernel-timing", default="on", choices=["on", "off"],
                    help="HIP events around every extend/shade launch of the timed steps (roofline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lit-parity", action="store_true", help="C4: skip the lit stand-in parity leg")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the CPUs this process may use, capped by the "
                                                                   "box's share (cgroup quota / OMP_NUM_THREADS)")
    ap.add_argument("--cpu-msamples", type=float, default=600.0,
                    help="size of the CPU-baseline row sample (Msamples of oracle work)")
    ap.add_argument("--alt-steps", "--f64-steps", type=int, default=10, dest="alt_steps",
                    help="after the headline run, time this many frames of the other precision on the same "
                         "config (f32 after an f64 headline and vice versa); 0 = skip")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    scene_name, width, aspect, spp, depth = CONFIGS[args.config]
    asset = sponza_asset()[1] if scene_name == "sponza" else None
    if scene_name.startswith("skybox"):  # the reference's earthmap.jpg (its bathroom.exr: no EXR decoder, magenta)
        os.environ.setdefault("RT_ASSETS", os.path.join(REPO, "tests", "golden", "assets"))
        asset = "the reference's assets/earthmap.jpg; bathroom.exr is not decodable (tinyexr absent): magenta skybox"
    # the scene exactly as the drop-in camera::render flattens it (C++ plugin surface, main.cc:198-225)
    cs = plugin.ConfigScene(scene_name, width, aspect)
    cam = cs.cam
    W, H = cam.image_width, cam.image_height
    prec = abi.RT_PREC_F64 if args.precision == "f64" else abi.RT_PREC_F32

    ctx = rt_amd.Context(local)
    ctx.upload(cs.desc)
    # the frame's 16x16 tiles dealt round-robin over the ranks, gathered to rank 0 (rt_amd.distributed)
    shard = FrameSharding(W, H, world, rank, dev)
    counts = shard.counts

    copy_stream = torch.cuda.Stream(dev)
    copy_h = copy_stream.cuda_stream
    hip = Hip()

    def run(precision, steps, warmup, timing):
        """warmup + `steps` timed frames; returns (elapsed s (max over ranks), stats, rank 0's host framebuffer
        of the last frame)."""
        tdtype = torch.float64 if precision == abi.RT_PREC_F64 else torch.float32
        out, fb = shard.buffers(tdtype)
        params = ctx.params(spp, depth, args.seed, precision, samples_per_item=args.chunk, pool_slots=args.pool,
                            segments_per_launch=args.segments_per_launch,
                            traversal=abi.RT_TRAV_ORDERED if args.traversal == "ordered" else abi.RT_TRAV_AUTO)
        # a step ends with the complete linear framebuffer in rank 0's host memory. Two device
        # framebuffers and two pinned host buffers: frame i's D2H runs on a copy stream while frame i + 1
        # renders, so only the last frame's copy is exposed; a buffer's next scatter waits for its last copy.
        fbs = [fb, torch.zeros_like(fb)] if rank == 0 else [None, None]
        hosts = [torch.empty(fb.shape, dtype=tdtype, pin_memory=True) for _ in range(2)] if rank == 0 else None
        nstep = [0]
        # the copies and their ordering by HIP calls (events made once): torch's per-call event and stream
        # objects cost ~1 ms of host time per frame, more than C1's whole 0.6 ms frame
        cur_h = torch.cuda.current_stream(dev).cuda_stream
        ready = [hip.event() for _ in range(2)]
        copied = [hip.event() for _ in range(2)]
        used = [False, False]
        nbytes = fb.numel() * fb.element_size() if rank == 0 else 0

        def step():
            k = nstep[0] % 2
            nstep[0] += 1
            if used[k]:
                hip.wait(cur_h, copied[k])
            # render this rank's tiles on torch's current stream (the default = the HIP null stream); the
            # RCCL gather and rank 0's scatter are queued behind it on the same stream
            shard.frame(ctx, cam, params, out, fbs[k])
            if rank == 0:
                hip.record(ready[k], cur_h)
                hip.wait(copy_h, ready[k])
                hip.d2h(hosts[k].data_ptr(), fbs[k].data_ptr(), nbytes, copy_h)
                hip.record(copied[k], copy_h)
                used[k] = True

        for _ in range(warmup):
            step()
        ctx.set_timing(timing)
        ctx.reset_counters()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            step()  # stream-ordered: the host enqueues the next frame while the GPU renders this one
        torch.cuda.synchronize(dev)  # every stream of the device: the last frame's D2H included
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        st = ctx.stats()  # totals over the timed steps (kernel time from HIP events on the render stream)
        ctx.set_timing(False)
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, st, (hosts[(nstep[0] - 1) % 2] if rank == 0 else None)

    elapsed, st, fb = run(prec, args.steps, args.warmup, args.kernel_timing == "on")
    segs, step_ms, iters = st.segments, st.step_ms, st.iterations
    segs_total = float(segs)
    if world > 1:
        s = torch.tensor([segs], dtype=torch.float64, device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        segs_total = float(s.item())
    total_samples = W * H * spp * args.steps
    value = total_samples / elapsed / 1e6
    kern = "k_step" if args.segments_per_launch > 0 else "k_persist"
    alt_name = "f32" if args.precision == "f64" else "f64"
    alt_prec = abi.RT_PREC_F32 if alt_name == "f32" else abi.RT_PREC_F64
    alt_run = None
    if args.alt_steps > 0:
        alt_run = run(alt_prec, args.alt_steps, 1, args.kernel_timing == "on")

    if rank == 0:
        my_samples = counts[0] * spp * args.steps
        seg_per_sample = segs / max(1, my_samples)
        key = workload_key(scene_name, W, H, spp, depth, args)
        # dominant kernel of rank 0 (k_persist: the persistent extend+shade loop, one launch per frame;
        # k_step with --segments-per-launch K: the fused wavefront step), average launch duration from HIP
        # events on the render stream. It is VALU-issue bound: path state stays in registers, so HBM
        # moves ~0.1 % of the classic wavefront's bytes. achieved = VALU work per launch (rocprofv3
        # counters of this build and workload, profiles/*_pmc.json) / live launch time.
        roof = None
        if args.kernel_timing == "on":
            roof = roofline(key, st, segs, my_samples, elapsed, kern, prec == abi.RT_PREC_F64)
        cpu = parity = None
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or cpu_threads()[0]
            # C4: lit 16x16 tiles (the reference's x-median tree renders ~2 rows of the stand-in in the
            # budget, and those rows are near-black); the other configs: evenly spaced full rows
            sample = lit_tiles(fb, W, H) if scene_name == "sponza" else None
            cpu, ptiles, ref_px = cpu_baseline(scene_name, width, aspect, spp, depth, args.seed, threads,
                                               args.cpu_msamples, tiles=sample)
            if scene_name == "sponza":
                cpu["baseline_tree"] = "x-median (bvh_node.h:13-47): the reference's own build, not the SAH tree"
            parity = parity_tiles(fb, W, ptiles, ref_px, rel_tol=1e-9 if prec == abi.RT_PREC_F64 else None)
        alt_line = None
        if alt_run is not None:
            ea, sta, fba = alt_run
            va = W * H * spp * args.alt_steps / ea / 1e6
            sa = sta.segments / max(1, counts[0] * spp * args.alt_steps)
            alt_line = {"value": round(va, 2), "unit": "Msamples/s", "steps": args.alt_steps,
                        "ms_per_step": round(ea / args.alt_steps * 1e3, 3),
                        "dtype": "fp64" if alt_name == "f64" else "fp32", "segments_per_sample": round(sa, 4),
                        "note": ("the same frames on the fp32 production path (north_star: per-channel RMSE < 1e-4 "
                                 "against the fp64 reference), timed the same way after the headline run"
                                 if alt_name == "f32" else
                                 "the same frames on the fp64 path (the reference's precision, vec3.h:7), timed "
                                 "the same way after the headline run")}
            if args.kernel_timing == "on":
                alt_line["roofline"] = roofline(workload_key(scene_name, W, H, spp, depth, args, alt_name), sta,
                                                sta.segments, counts[0] * spp * args.alt_steps, ea, kern,
                                                alt_name == "f64")
            if cpu:
                alt_line["parity"] = parity_tiles(fba, W, ptiles, ref_px, rel_tol=1e-9 if alt_name == "f64" else None)
                tree = "baseline_tree" in cpu  # (C4: see the headline object's ratio_vs_reference_tree)
                alt_line["ratio_vs_reference_tree" if tree else "speedup_vs_cpu_baseline"] = round(va / cpu["value"], 1)
                alt_line["ratio_vs_reference_tree_per_segment" if tree else "speedup_per_segment"] = round(
                    va * sa / (cpu["value"] * cpu["segments_per_sample"]), 1)
        lit = None
        if cpu and scene_name == "sponza" and not args.no_lit_parity:
            lit = lit_parity(ctx, width, aspect, spp, depth, args.seed, threads,
                             [prec] + ([alt_prec] if alt_run is not None else []))
        line = {
            "metric": "Msamples/sec (pixels*spp) Cornell Box 800x800@1024spp; 1/2/4/8-GPU scaling"
            if args.config == "c2" else f"Msamples/sec (pixels*spp) {scene_name} {W}x{H}@{spp}spp",
            "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "fp32" if prec == abi.RT_PREC_F32 else "fp64",
            "data": asset or "synthetic (the reference's scene, procedurally built; no assets)",
            "config": {"workload": f"{scene_name} {W}x{H} {spp}spp depth {depth}, light sampling on",
                       "key": key, "src_sha": buildinfo.src_sha(),
                       "image": [W, H], "spp": spp, "max_depth": depth, "tiles": "16x16 round-robin over ranks",
                       "parallelism": f"tiles{world}", "segments_per_sample": round(seg_per_sample, 4),
                       "segments_total": segs_total / args.steps, "kernel_timing": args.kernel_timing,
                       "rounds_per_frame": iters // max(1, args.steps), "grid_lanes": st.grid_lanes,
                       "timed_region": "barrier + sync .. sync + barrier around the steps; a step ends with the "
                                       "whole linear framebuffer in rank 0's pinned host memory (its D2H on a "
                                       "copy stream, overlapped with the next frame's render; the last one "
                                       "inside the region); parity reads that host copy"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity": parity,
            alt_name: alt_line,
        }
        if lit is not None:
            line["lit_parity"] = lit
        if cpu:
            line["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
            # per unit of work: the GPU stops zero-throughput paths, the oracle does not, so
            # it traces more segments per sample
            line["speedup_per_segment"] = round(value * seg_per_sample / (cpu["value"] * cpu["segments_per_sample"]),
                                                1)
            if "baseline_tree" in cpu:
                # the CPU baseline runs the reference's own x-median tree over 262k triangles (bvh_node.h:13-47), the
                # GPU a SAH tree: the ratio compares trees as much as hardware, so it is not reported as a speedup
                line["ratio_vs_reference_tree"] = line.pop("speedup_vs_cpu_baseline")
                line["ratio_vs_reference_tree_per_segment"] = line.pop("speedup_per_segment")
                line["speedup_baseline_tree"] = "x-median (bvh_node.h:13-47): not a like-for-like speedup"
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
