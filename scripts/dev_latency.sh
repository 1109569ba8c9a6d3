# Development: memory-latency counters of one bench frame.  bash scripts/dev_latency.sh <cfg> [bench args]
set -e
export TMPDIR=/tmp
cfg=$1; shift
out=gpurun_out/lat/$cfg; mkdir -p $out
B="bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --f64-steps 0 --kernel-timing off $*"
timeout -s KILL 90 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES -d $out/a -o run --output-format csv -- python3 $B > $out/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $out/b -o run --output-format csv -- python3 $B > $out/b.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH_LEVEL SQ_IFETCH SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $out/c -o run --output-format csv -- python3 $B > $out/c.log 2>&1
python3 - $out <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float)
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "persist" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(tot): print(k, "%.4g" % tot[k])
for a, b in [("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM_RD"), ("SQ_INST_LEVEL_SMEM", "SQ_INSTS_SMEM"), ("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS")]:
    if tot[b]: print(a, "/", b, "%.1f" % (tot[a] / tot[b]))
PY
