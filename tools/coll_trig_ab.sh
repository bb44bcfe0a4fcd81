#!/bin/bash
# A/B of exact vs hardware trig in the specialised collision kernels (KINHIP_COLL_FAST_TRIG), interleaved
set -u
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 0 1; do
    KINHIP_COLL_FAST_TRIG=$v timeout -k 10 300 python bench.py --no-cpu --steps 30 > gpurun_out/ct_$v.json 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/ct_$v.json').read().strip().splitlines()[-1]); c=d['config5_fk_sdf']
print('fast_trig=$v', {k: round(v['avg_launch_us'], 1) for k, v in c.items() if isinstance(v, dict)})"
  done
done
