#!/bin/bash
# A/B of the SLP vectoriser in the run-time specialised kernels (KINHIP_JIT_SLP: packed v_pk_* fp32
# operations), interleaved, two rounds of bench.py --no-cpu.
set -e
mkdir -p gpurun_out
for r in 1 2; do for v in 0 1; do
  KINHIP_JIT_SLP=$v timeout -k 10 300 python bench.py --no-cpu --steps 30 > gpurun_out/slp_${v}_$r.json 2>/dev/null
  echo "slp=$v round $r done"
done; done
