#!/bin/bash
# GPU box: kernel trace + PMC passes of one bench frame (+1 warmup), then the summaries into profiles/.
#   scripts/prof_pmc.sh <outdir> <tag> [bench args]
# Counters follow MI355X_MICROARCH.md: --pmc passes alone (no sys/runtime trace), FETCH_SIZE and
# WRITE_SIZE in separate passes.
set -e
out=$1; tag=$2; shift 2
export TMPDIR=/tmp
mkdir -p $out
B="bench.py --steps 1 --warmup 1 --no-cpu-baseline --f64-steps 0 --kernel-timing off $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $B > $out/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d $out/pmc1 -o run --output-format csv -- python3 $B > $out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $out/pmc2 -o run --output-format csv -- python3 $B > $out/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS -d $out/pmc3 -o run --output-format csv -- python3 $B > $out/pmc3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $out/pmc4 -o run --output-format csv -- python3 $B > $out/pmc4.log 2>&1
# the VALU instruction mix: fp64 instructions issue at half the fp32 rate (bench.py's fp64 roofline)
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 -d $out/pmc5 -o run --output-format csv -- python3 $B > $out/pmc5.log 2>&1
# conversions and 64-bit integer instructions (bench.py's VALU issue-cycle model: 4 cycles each)
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT -d $out/pmc6 -o run --output-format csv -- python3 $B > $out/pmc6.log 2>&1
# the memory pipeline: TA / TD busy cycles and L1 (TCP) accesses against the GPU's active cycles (C4's bound)
timeout -k 10 300 rocprofv3 --pmc TA_TA_BUSY TD_TD_BUSY TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ GRBM_GUI_ACTIVE -d $out/pmc7 -o run --output-format csv -- python3 $B > $out/pmc7.log 2>&1
key=$(python3 -c "import json; print([json.loads(l) for l in open('$out/trace.log') if l.startswith('{\"metric')][-1]['config']['key'])")
python3 scripts/pmc_summary.py $out $tag "$key" $out/summary
