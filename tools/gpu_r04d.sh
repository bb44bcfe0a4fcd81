# round-4 session D: config-4 IK A/B -- the fp64 damped solve inside the fp32 kernel (KINHIP_IK_F64SOLVE) and
# the solver settings (fixed lambda / max_step 0.5 against lambda^2 + 0.01|e|^2 / max_step 1)
mkdir -p gpurun_out
export AB_F32=1
timeout -k 10 500 python -u tools/ab.py ik --reps 2 base IK_DAMP=0.01,IK_MAXSTEP=1.0 \
  "KINHIP_JIT_DEFS=-DKINHIP_IK_F64SOLVE=0" "KINHIP_JIT_DEFS=-DKINHIP_IK_F64SOLVE=0,IK_DAMP=0.01,IK_MAXSTEP=1.0" \
  IK_MAXSTEP=1.0 IK_DAMP=0.01 > gpurun_out/r04d_ik_ab.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04d_ik_ab.txt; exit $rc
