#!/bin/bash
# GPU box: measured issue cost of single VALU opcodes (tools/valu_rates), and how the SQ counters count
# them (two --pmc passes of the same program).   scripts/valu_rates.sh <outdir>
set -e
out=$1
export TMPDIR=/tmp
mkdir -p $out
timeout -k 10 120 tools/valu_rates > $out/rates.json
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_WAVE_CYCLES -d $out/pmcA -o run --output-format csv -- tools/valu_rates > $out/pmcA.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU -d $out/pmcB -o run --output-format csv -- tools/valu_rates > $out/pmcB.log 2>&1
python3 - $out <<'PY'
import csv, glob, json, re, sys
from collections import defaultdict
out = sys.argv[1]
rates = json.load(open(out + "/rates.json"))
names = list(rates["ops"])
per = defaultdict(dict)  # opcode -> counter -> value of the second (warm) dispatch
for p in ("pmcA", "pmcB"):
    seen = defaultdict(int)
    rows = []
    for f in glob.glob(f"{out}/{p}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    disp = {}
    for r in rows:
        m = re.search(r"k_rate<(\d+)>", r["Kernel_Name"])
        if not m:
            continue
        disp.setdefault((int(r["Dispatch_Id"]), int(m.group(1))), defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
    cnt = defaultdict(int)
    for (d, k), c in sorted(disp.items()):
        cnt[k] += 1
        if cnt[k] == 2:
            per[names[k]].update(c)
instr = rates["cus"] * 4 * rates["waves_per_simd"] * rates["instr_per_wave"]
res = {"per_wave_instr": rates["ops"], "unit": rates["unit"], "counters_per_instr": {}}
for n in names:
    c = per.get(n, {})
    res["counters_per_instr"][n] = {k: round(v / instr, 3) for k, v in sorted(c.items())}
json.dump(res, open(out + "/valu_rates.json", "w"), indent=1)
print(json.dumps({k: v["cycles"] for k, v in res["per_wave_instr"].items()}))
PY
