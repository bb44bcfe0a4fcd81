# round-4 session G: IK solve variants (fp64 solve / fp32 / fp32 + fp64-residual refinement: speed, and the
# fp32 bound test on the refinement), the probe's occupancy sweep, the ld = N store-path knobs
mkdir -p gpurun_out
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
( AB_F32=1 timeout -k 10 400 python -u tools/ab.py ik --reps 2 base "KINHIP_JIT_DEFS=-DKINHIP_IK_F64SOLVE=2" \
    "KINHIP_JIT_DEFS=-DKINHIP_IK_F64SOLVE=0" \
 && KINHIP_LIB=$AB KINHIP_JIT_DEFS=-DKINHIP_IK_F64SOLVE=2 timeout -k 10 300 python -u -m pytest \
    tests/test_gpu_ik_fp32_bound.py -m gpu -v -s --timeout 200 --timeout-method thread 2>&1 | grep -E "fp32 step|passed|failed|Error" \
 && timeout -k 10 300 python -u tools/probe_occ.py \
 && timeout -k 10 400 python -u tools/ab.py jl --reps 2 base KINHIP_FK_PER_LANE=2 "KINHIP_JIT_DEFS=-DKINHIP_STORE_AUX=0" \
    KINHIP_FK_PER_LANE=4 ) > gpurun_out/r04g.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04g.txt; exit $rc
