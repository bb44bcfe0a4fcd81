#!/bin/bash
set -u
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
for cut in 10 0; do
  echo "== hand-over at $cut"
  timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_IK_P1_CUT=$cut KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=9 python -u tools/ik_timeline.py 2>&1 | grep -v amdgpu.ids || exit 1
done
