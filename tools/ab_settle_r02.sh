#!/bin/bash
# settle_loads A/B (KINHIP_SETTLE_LOADS via KINHIP_JIT_DEFS) on the collision and FK legs, after parity.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_collision.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "coll or fk or specialized or golden" > gpurun_out/ab_settle_tests.log 2>&1 \
  || { tail -40 gpurun_out/ab_settle_tests.log; exit 1; }
tail -1 gpurun_out/ab_settle_tests.log
for rep in 1 2; do
  for v in 1 0; do
    timeout -k 10 120 env KINHIP_JIT_DEFS="-DKINHIP_SETTLE_LOADS=$v" python tools/coll_spec_ab.py 2>/dev/null | sed "s/^/settle=$v /" || exit 1
    timeout -k 10 120 env KINHIP_JIT_DEFS="-DKINHIP_SETTLE_LOADS=$v" python tools/fk_legs_ab.py 2>/dev/null | sed "s/^/settle=$v /" || exit 1
  done
done
