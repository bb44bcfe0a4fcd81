#!/bin/bash
# IK tests, config-4 timing (product) x2, timeline with the hand-over
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ik_rpy.py tests/test_gpu_collision_ik.py \
  -m gpu -x -q -k "ik" --timeout 300 --timeout-method thread > gpurun_out/r03_ik_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03_ik_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do timeout -k 10 120 env AB_SPEC=1 IK_N=65536 python -u tools/ik_ab.py 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 120 env AB_SPEC=1 IK_N=1048576 AB_F32=1 python -u tools/ik_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 env KINHIP_LIB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=9 python -u tools/ik_timeline.py 2>&1 | grep -v "amdgpu.ids\|iters "
