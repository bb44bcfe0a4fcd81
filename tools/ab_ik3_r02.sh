#!/bin/bash
# IK two-phase schedule (KINHIP_IK_TWO_PHASE: unset = automatic, 0 = off, 1 = forced) after the IK parity tests.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_collision_ik.py tests/test_dist_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "ik or nakamura or dist" > gpurun_out/ab_ik_tests.log 2>&1 \
  || { tail -40 gpurun_out/ab_ik_tests.log; exit 1; }
tail -1 gpurun_out/ab_ik_tests.log
for rep in 1 2; do
  for v in auto 0 1; do
    for n in 32768 65536 262144; do
      if [ $v = auto ]; then e=""; else e="KINHIP_IK_TWO_PHASE=$v"; fi
      timeout -k 10 120 env $e AB_SPEC=1 IK_N=$n python tools/ik_ab.py 2>/dev/null | sed "s/^/two=$v n=$n /" || exit 1
    done
  done
done
