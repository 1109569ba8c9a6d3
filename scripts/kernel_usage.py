#!/usr/bin/env python3
"""Registers, spills and occupancy of the persistent kernels from a -Rpass-analysis=kernel-resource-usage
compile log:  python scripts/kernel_usage.py <log> [substring filter]"""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read()
filt = sys.argv[2] if len(sys.argv) > 2 else "k_persist"
for b in re.split(r"remark: [^\n]*Function Name: ", txt)[1:]:
    name = b.split("\n")[0].split()[0]
    dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    dn = dn.replace("(anonymous namespace)::", "").replace("void ", "")
    if filt not in dn:
        continue

    def g(k):
        m = re.search(k + r": (\d+)", b)
        return m.group(1) if m else "?"
    v, a, sc = g("VGPRs"), g("AGPRs"), g(r"ScratchSize \[bytes/lane\]")
    w, sg = g(r"Occupancy \[waves/SIMD\]"), g("SGPRs")
    print(f"vgpr {v:>3} agpr {a:>2} scratch {sc:>3} waves {w} sgpr {sg:>3}  {dn.split('(')[0]}")
