#!/bin/bash
# dev helper (GPU box): kernel trace + PMC passes for one C2 frame. Usage: scripts/prof_pmc.sh <outdir> [bench args]
set -e
out=$1; shift
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --kernel-timing off $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- $B > $out/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -d $out/pmc1 -o run --output-format csv -- $B > $out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $out/pmc2 -o run --output-format csv -- $B > $out/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS -d $out/pmc3 -o run --output-format csv -- $B > $out/pmc3.log 2>&1
