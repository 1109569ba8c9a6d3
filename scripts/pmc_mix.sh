#!/bin/bash
# GPU box: the VALU instruction mix of one bench frame (one --pmc pass; counters within the SQ block limit)
#   scripts/pmc_mix.sh <outdir> [bench args]      -> <outdir>/mix.txt (per-launch means of the dominant kernel)
set -e
out=$1; shift
export TMPDIR=/tmp
mkdir -p $out
B="bench.py --steps 1 --warmup 1 --no-cpu-baseline --f64-steps 0 --kernel-timing off $*"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INST_CYCLES_SALU -d $out/mix -o run --output-format csv -- python3 $B > $out/mix.log 2>&1
python3 - $out <<'PY'
import csv, glob, sys
from collections import defaultdict
tot = defaultdict(float); n = defaultdict(int)
for f in glob.glob(sys.argv[1] + "/mix/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_persist" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
with open(sys.argv[1] + "/mix.txt", "w") as fh:
    for k in sorted(tot):
        fh.write(f"{k} {tot[k]:.4g} (entries {n[k]})\n")
print(open(sys.argv[1] + "/mix.txt").read())
PY
