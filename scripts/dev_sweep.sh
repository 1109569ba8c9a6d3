#!/bin/bash
# Development sweep on the GPU box: bench variants (library builds, K, pool) on C2, one line each.
#   scripts/dev_sweep.sh <out dir> ["<label>|<env assignments>|<bench args>" ...]
out=$1; shift
mkdir -p $out
for spec in "$@"; do
  IFS='|' read -r label envs args <<< "$spec"
  env $envs timeout -k 10 120 python bench.py --no-cpu-baseline $args > $out/$label.log 2>&1 || { echo "$label failed"; exit 1; }
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$out/$label.log') if l.startswith('{')][-1]; print('$label', d['value'], d['roofline']['avg_launch_us'] if d['roofline'] else '')"
done
