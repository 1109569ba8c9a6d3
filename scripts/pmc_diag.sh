#!/bin/bash
# GPU box: memory-pipeline utilisation of one bench frame (one --pmc pass within the block limits: 2 TA,
# 2 TD, 4 TCP, 2 GRBM): TA / TD busy cycles, L1 (TCP) accesses and L2 read requests, against the GPU's
# active cycles.   scripts/pmc_diag.sh <outdir> [bench args]   -> <outdir>/diag.json
set -e
out=$1; shift
export TMPDIR=/tmp
mkdir -p $out
B="bench.py --steps 1 --warmup 1 --no-cpu-baseline --f64-steps 0 --kernel-timing off $*"
timeout -k 10 300 rocprofv3 --pmc TA_TA_BUSY TD_TD_BUSY TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_TCP_TA_DATA_STALL_CYCLES GRBM_GUI_ACTIVE -d $out/diag -o run --output-format csv -- python3 $B > $out/diag.log 2>&1
python3 - $out <<'PY'
import csv, glob, json, sys
from collections import defaultdict
out = sys.argv[1]
acc = defaultdict(list)
for f in glob.glob(out + "/diag/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_persist" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
gui = m.get("GRBM_GUI_ACTIVE", 0) / 8  # per-XCD active cycles
res = {"per_launch_means": m,
       "ta_busy_frac": m.get("TA_TA_BUSY", 0) / (256 * gui) if gui else None,
       "td_busy_frac": m.get("TD_TD_BUSY", 0) / (256 * gui) if gui else None,
       "tcp_accesses_per_cu_cycle": m.get("TCP_TOTAL_CACHE_ACCESSES", 0) / (256 * gui) if gui else None,
       "note": "TA/TD busy summed over the 256 CUs' units, against GRBM_GUI_ACTIVE / 8 XCDs"}
json.dump(res, open(out + "/diag.json", "w"), indent=1)
print(json.dumps(res))
PY
