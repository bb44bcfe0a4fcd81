#!/bin/bash
# IK iteration sections (tools/ik_sect.py) for k = 0 (no stamps: the lane total is not measured) .. 7
set -u
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
for k in 1 2 3 4 5 6 7; do
  timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=$k python -u tools/ik_sect.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for k in 1 3; do
  timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=$k IK_N=262144 python -u tools/ik_sect.py 2>&1 | grep -v amdgpu.ids || exit 1
done
