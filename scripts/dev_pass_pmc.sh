#!/bin/bash
# GPU box, development: a few counters of C4 fp64 at one and at three chunk passes (render() budget).
export TMPDIR=/tmp
out=$1; shift
mkdir -p $out
B="bench.py --config c4 --precision f64 --steps 1 --warmup 0 --no-cpu-baseline --alt-steps 0 --kernel-timing off"
for b in 8000000000 1073741824; do
  RT_PARTIAL_BUDGET=$b timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $out/p1_$b -o run --output-format csv -- python3 $B > $out/p1_$b.log 2>&1 || exit 1
  RT_PARTIAL_BUDGET=$b timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES GRBM_GUI_ACTIVE TCP_TCC_READ_REQ -d $out/p2_$b -o run --output-format csv -- python3 $B > $out/p2_$b.log 2>&1 || exit 1
done
