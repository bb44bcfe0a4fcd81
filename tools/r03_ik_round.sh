#!/bin/bash
# Round 3 IK iteration work: IK parity tests, the per-iteration probe, section stamps, config-4 timing
# over the phase-1 hand-over point (A/B build) and the product default.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ik_rpy.py tests/test_gpu_collision_ik.py \
  -m gpu -x -q -k "ik" --timeout 300 --timeout-method thread > gpurun_out/r03_ik_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_ik_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ik_iter_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/r03_ik_sect.sh || exit 1
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
for cut in 0 8 10 12; do
  timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_IK_P1_CUT=$cut AB_SPEC=1 IK_N=65536 python -u tools/ik_ab.py \
    2>&1 | grep -v amdgpu.ids | sed "s/^/cut=$cut /" || exit 1
done
timeout -k 10 120 env AB_SPEC=1 IK_N=65536 python -u tools/ik_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/product /"
