#!/bin/bash
set -u
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
for r in 1 2 3; do
for cut in 7 8 9 10 11 12; do
  timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_IK_P1_CUT=$cut AB_SPEC=1 IK_N=65536 python -u tools/ik_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/cut=$cut /" || exit 1
done
done
