#!/bin/bash
# IK: parity tests (oracle iterates, lanes / schedule identity, acceptance, bistage), then timings.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_collision_ik.py tests/test_dist_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "ik or nakamura or dist" > gpurun_out/ab_ik_tests.log 2>&1 \
  || { tail -40 gpurun_out/ab_ik_tests.log; exit 1; }
tail -1 gpurun_out/ab_ik_tests.log
for rep in 1 2; do
  for n in 65536 1048576; do
    timeout -k 10 120 env AB_SPEC=1 IK_N=$n python tools/ik_ab.py 2>/dev/null | sed "s/^/n=$n /" || exit 1
  done
  timeout -k 10 120 env AB_SPEC=0 AB_F32=1 IK_N=65536 python tools/ik_ab.py 2>/dev/null | sed "s/^/generic n=65536 /" || exit 1
done
