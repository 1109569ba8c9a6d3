# Development: automatic item sizes (RT_ITEM_* overrides) on C2 and C3, full frame vs one rank of eight.
#   bash scripts/dev_tail.sh
set -e
mkdir -p gpurun_out/tail
t() {  # name, env..., then the config
  local n=$1; shift
  env "$@" timeout -k 10 120 python3 scripts/dev_tail.py --config $CFG --chunks 0 > gpurun_out/tail/$n.log 2>&1
  python3 -c "
import json
for l in open('gpurun_out/tail/$n.log'):
    if l.startswith('{'):
        d = json.loads(l)
        if d['case'] != 'full_spp/8': print('$n', d['case'], d['kernel_ms'], d['msamples_s'])"
}
CFG=c2
t c2_uniform32 RT_ITEM_TAIL_FRAC=0
t c2_f125_t8 RT_ITEM_TAIL_FRAC=0.125
t c2_f25_t8 RT_ITEM_TAIL_FRAC=0.25
t c2_f375_t8 RT_ITEM_TAIL_FRAC=0.375
t c2_f25_t4 RT_ITEM_TAIL_FRAC=0.25 RT_ITEM_TAIL_CHUNK_FLAT=4
t c2_f25_t16 RT_ITEM_TAIL_FRAC=0.25 RT_ITEM_TAIL_CHUNK_FLAT=16
CFG=c3
t c3_uniform16 RT_ITEM_TAIL_FRAC=0
t c3_f25_t4 RT_ITEM_TAIL_FRAC=0.25
t c3_b8_f25_t4 RT_ITEM_CHUNK=8 RT_ITEM_TAIL_FRAC=0.25
t c3_b8_f25_t2 RT_ITEM_CHUNK=8 RT_ITEM_TAIL_FRAC=0.25 RT_ITEM_TAIL_CHUNK=2
t c3_b4_f0 RT_ITEM_CHUNK=4 RT_ITEM_TAIL_FRAC=0
t c3_b8_f5_t4 RT_ITEM_CHUNK=8 RT_ITEM_TAIL_FRAC=0.5
