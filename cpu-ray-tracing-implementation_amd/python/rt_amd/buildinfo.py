"""Identity of the device code a measurement was taken on.

bench.py reads per-launch PMC figures (VALU instructions, HBM bytes) from the committed
profiles/ summaries; a summary only applies to the build it was collected on, so both sides
key it by this hash of the HIP sources and the build flags.
"""
import glob
import hashlib
import os

from .abi import PKG_DIR, REPO_DIR


def src_sha():
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(PKG_DIR, "csrc", "*"))) + [os.path.join(REPO_DIR, "Makefile"),
                                                                      os.path.join(REPO_DIR, "include", "rt_hip.h")]
    for f in files:
        if os.path.isfile(f):
            h.update(os.path.basename(f).encode())
            with open(f, "rb") as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def host_cpu():
    """The host's CPU as the CPU baseline must state it: model, logical CPUs, the CPUs this
    process may run on, and the cgroup CPU quota (the box's share), if any."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    return {"model": model, "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "cgroup_quota_cpus": quota, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
