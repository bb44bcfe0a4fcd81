#!/bin/bash
# IK: a lane group skips one pass after taking a target (KINHIP_IK_FRESH_SKIP via KINHIP_JIT_DEFS), after parity.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_collision_ik.py tests/test_dist_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "ik or nakamura or dist" > gpurun_out/ab_ik_tests.log 2>&1 \
  || { tail -40 gpurun_out/ab_ik_tests.log; exit 1; }
tail -1 gpurun_out/ab_ik_tests.log
for rep in 1 2; do
  for v in 1 0; do
    for n in 65536 1048576; do
      timeout -k 10 120 env AB_SPEC=1 IK_N=$n KINHIP_JIT_DEFS="-DKINHIP_IK_FRESH_SKIP=$v" python tools/ik_ab.py 2>/dev/null \
        | sed "s/^/skip=$v n=$n /" || exit 1
    done
  done
done
