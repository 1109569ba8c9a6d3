#!/usr/bin/env python3
"""Summarise the rocprofv3 passes of scripts/prof_pmc.sh into profiles/.

  python scripts/pmc_summary.py <prof dir> <tag> <workload> [<output dir>]

Writes
  profiles/<tag>_kernel_stats.csv   the --kernel-trace --stats summary (copied as rocprofv3 wrote it)
  profiles/<tag>_pmc_summary.csv    per kernel and counter: dispatches, mean and total over the run
  profiles/<tag>_pmc.json           per-launch figures of the dominant kernel, keyed by workload and
                                    build (rt_amd.buildinfo.src_sha), read by bench.py for its roofline:
                                    SQ_INSTS_VALU (VALU-issue roofline) and HBM bytes (roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md (HBM [CDNA4]): FETCH_SIZE and WRITE_SIZE are in KiB,
and on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024. FETCH_SIZE and WRITE_SIZE come from
separate passes (they do not fit one pass), averaged over the same launches.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    # "void (anonymous namespace)::k_step<float, ...>((anonymous namespace)::Params<float>)" -> "k_step<float, ...>"
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0]


def main():
    prof, tag, workload = sys.argv[1], sys.argv[2], sys.argv[3]
    # summaries land in profiles/ (here), or in the given directory (on the GPU box: under gpurun_out/,
    # which gpurun copies back; then they are copied into profiles/ and committed)
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(REPO, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(prof, "trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(out, f"{tag}_kernel_stats.csv"))
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per dispatch)
    for f in sorted(glob.glob(os.path.join(prof, "pmc*", "*counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    rows = []
    for k, counters in sorted(acc.items()):
        for c, v in sorted(counters.items()):
            rows.append([k, c, len(v), sum(v) / len(v), sum(v)])
    with open(os.path.join(out, f"{tag}_pmc_summary.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "counter", "dispatches", "mean", "total"])
        w.writerows(rows)
    # the dominant kernel: all k_persist (default schedule) or k_step instantiations of the run
    fam = "k_persist" if any(k.startswith("k_persist") for k in acc) else "k_step"
    fetch, write, traffic = [], [], None
    for k, counters in acc.items():
        if k.startswith(fam):
            fetch += counters.get("FETCH_SIZE", [])
            write += counters.get("WRITE_SIZE", [])
    if fetch and write:
        f_mean, w_mean = sum(fetch) / len(fetch), sum(write) / len(write)
        traffic = {"kernel": fam, "workload": workload, "launches_fetch_pass": len(fetch),
                   "launches_write_pass": len(write), "fetch_size_kib_mean": f_mean, "write_size_kib_mean": w_mean,
                   "bytes_per_launch": (2.0 * f_mean + w_mean) * 1024.0,
                   "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (KiB; gfx950 FETCH_SIZE counts half, "
                              "MI355X_MICROARCH.md HBM [CDNA4])", "source": f"{tag}_pmc_summary.csv"}
        print(json.dumps(traffic))
    # everything bench.py's roofline needs, per launch of the dominant kernel family
    def fam_mean(c):
        v = [x for k, cs in acc.items() if k.startswith(fam) for x in cs.get(c, [])]
        return (sum(v) / len(v), len(v)) if v else (None, 0)
    valu, nv = fam_mean("SQ_INSTS_VALU")
    gui, _ = fam_mean("GRBM_GUI_ACTIVE")
    # the dominant kernel instantiation (longest total time in the kernel trace) and its static VALU opcode
    # mix (scripts/valu_static_mix.py), for bench.py's issue-cycle model
    mix_file = None
    trace_avg = None
    if stats:
        with open(stats[0]) as fh:
            top = max(csv.DictReader(fh), key=lambda r: float(r["TotalDurationNs"]))
        trace_avg = float(top["AverageNs"])
        kname = top["Name"][5:] if top["Name"].startswith("void ") else top["Name"]
        kname = kname.split("((anonymous namespace)::Params")[0]
        sys.path.insert(0, os.path.join(REPO, "scripts"))
        import subprocess
        lib = os.environ.get("RT_HIP_LIB") or os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "build",
                                                          "librt_hip.so")
        mix_file = f"{tag}_valu_mix.json"
        subprocess.run([sys.executable, os.path.join(REPO, "scripts", "valu_static_mix.py"), lib, kname, "--out",
                        os.path.join(out, mix_file)], check=True)
    if valu is not None:
        sys.path.insert(0, os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python"))
        from rt_amd import buildinfo
        d = {"workload": workload, "src_sha": buildinfo.src_sha(), "kernel": fam, "launches": nv,
             "valu_per_launch": valu,
             "valu_issue_frac_measured_clock": round(valu * 2 / (1024 * gui / 8), 4) if gui else None,
             "grbm_gui_active_per_launch": gui,
             # the dominant kernel's average duration in the --kernel-trace pass, and the shader clock the
             # profiled launches ran at: GPU-active cycles per XCD (GRBM_GUI_ACTIVE / 8) over that duration
             "trace_avg_ns": trace_avg,
             "profiled_clock_ghz": round(gui / 8 / trace_avg, 4) if gui and trace_avg else None,
             # active lanes per issued VALU instruction (rocprof's VALUUtilization)
             "valu_lane_util": (round(fam_mean("SQ_THREAD_CYCLES_VALU")[0] / (64 * fam_mean("SQ_ACTIVE_INST_VALU")[0]), 4)
                                if fam_mean("SQ_THREAD_CYCLES_VALU")[0] and fam_mean("SQ_ACTIVE_INST_VALU")[0] else None),
             "wait_frac": (round(fam_mean("SQ_WAIT_ANY")[0] / fam_mean("SQ_WAVE_CYCLES")[0], 4)
                           if fam_mean("SQ_WAIT_ANY")[0] and fam_mean("SQ_WAVE_CYCLES")[0] else None),
             "hbm_bytes_per_launch": traffic["bytes_per_launch"] if fetch and write else None,
             "valu_mix": mix_file,
             # the L1 address path (TA): busy cycles of the 256 CUs' TA units over the GPU's active cycles
             "ta_busy_frac": (round(fam_mean("TA_TA_BUSY")[0] / (256 * gui / 8), 4)
                              if fam_mean("TA_TA_BUSY")[0] and gui else None),
             "tcp_accesses_per_launch": fam_mean("TCP_TOTAL_CACHE_ACCESSES")[0],
             "counters": {c: fam_mean(c)[0] for c in sorted({c for k, cs in acc.items() if k.startswith(fam)
                                                             for c in cs})},
             "formulas": {"valu_issue_frac_measured_clock": "SQ_INSTS_VALU * 2 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8 "
                                                            "XCDs)",
                          "valu_lane_util": "SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)",
                          "wait_frac": "SQ_WAIT_ANY / SQ_WAVE_CYCLES", "hbm_bytes": "(2*FETCH_SIZE + WRITE_SIZE) * 1024"},
             "source": f"{tag}_pmc_summary.csv"}
        with open(os.path.join(out, f"{tag}_pmc.json"), "w") as fh:
            json.dump(d, fh, indent=1)
        print(json.dumps(d))


if __name__ == "__main__":
    main()
