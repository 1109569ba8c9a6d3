#!/bin/bash
# dev helper: sweep segments-per-launch and pool size on the GPU box
for k in 1 2 4 8 16; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --segments-per-launch $k --steps 2 || exit 1
done
for pool in 524288 2097152; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --pool $pool --steps 2 || exit 1
done
