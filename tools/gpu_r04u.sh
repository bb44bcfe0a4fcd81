# round-4 session U: door sweep at a forced 5 waves per SIMD; config-4 phase-1 cut sweep (fixed / damped)
set -o pipefail
mkdir -p gpurun_out
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
( for w in 0 5 0 5; do
    KINHIP_LIB=$AB KINHIP_JIT_COLL_WAVES=$w timeout -k 10 200 python -u tools/scene_ab.py 15 | sed "s/^/waves=$w: /" || exit 1
  done
  AB_F32=1 timeout -k 10 500 python -u tools/ab.py ik --reps 2 base KINHIP_IK_P1_CUT=8 KINHIP_IK_P1_CUT=12 KINHIP_IK_P1_CUT=14 \
      IK_DAMP=0.01,IK_MAXSTEP=1.0 IK_DAMP=0.01,IK_MAXSTEP=1.0,KINHIP_IK_P1_CUT=8 IK_DAMP=0.01,IK_MAXSTEP=1.0,KINHIP_IK_P1_CUT=12 \
      IK_DAMP=0.01,IK_MAXSTEP=1.0,KINHIP_IK_P1_CUT=14 ) > gpurun_out/r04u.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04u.txt | tail -40; exit $rc
