# round-4 session M: config-4 per-lane timelines (fixed lambda vs the error-scaled damping)
mkdir -p gpurun_out
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
( KINHIP_LIB=$AB KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=9 timeout -k 10 200 python -u tools/ik_timeline.py \
 && IK_DAMP=0.01 IK_MAXSTEP=1.0 KINHIP_LIB=$AB KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=9 timeout -k 10 200 python -u tools/ik_timeline.py \
 ) > gpurun_out/r04m.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04m.txt; exit $rc
