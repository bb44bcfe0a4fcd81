#!/bin/bash
# Round 3: IK early hand-over (IkArgsT::p1_cut) -- the IK parity tests, then config-4 timings of the
# A/B build over the hand-over point (KINHIP_IK_P1_CUT; 0 = the round-2 schedule), two rounds.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ik_rpy.py -m gpu -x -q -k "ik" \
  --timeout 300 --timeout-method thread > gpurun_out/r03_ik_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_ik_tests.log; [ $rc -eq 0 ] || exit $rc
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
for r in 1 2; do
  for cut in 0 6 7 8 9 10 12; do
    timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_IK_P1_CUT=$cut AB_SPEC=1 AB_F32=1 IK_N=65536 python -u tools/ik_ab.py \
      2>&1 | grep -v amdgpu.ids | sed "s/^/cut=$cut /" || exit 1
  done
done
timeout -k 10 120 env AB_SPEC=1 IK_N=65536 python -u tools/ik_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/product /"
