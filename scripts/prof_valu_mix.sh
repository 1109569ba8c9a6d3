#!/bin/bash
# GPU box: one rocprofv3 --pmc pass of the VALU instruction mix (fp32 / fp64 add, mul, fma,
# transcendental) of one bench frame; output under <outdir>/pmc5 (scripts/pmc_summary.py reads it).
#   scripts/prof_valu_mix.sh <outdir> [bench args]
set -e
out=$1; shift
export TMPDIR=/tmp
mkdir -p $out
B="bench.py --steps 1 --warmup 1 --no-cpu-baseline --f64-steps 0 --kernel-timing off $*"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 -d $out/pmc5 -o run --output-format csv -- python3 $B > $out/pmc5.log 2>&1
