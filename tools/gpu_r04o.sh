# round-4 session O: phase-2 work spread over all CUs (A/B) and the IK schedule tests
mkdir -p gpurun_out
( AB_F32=1 timeout -k 10 400 python -u tools/ab.py ik --reps 2 base KINHIP_IK_P2_SPREAD=0 IK_DAMP=0.01,IK_MAXSTEP=1.0 \
    IK_DAMP=0.01,IK_MAXSTEP=1.0,KINHIP_IK_P2_SPREAD=0 \
 && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "ik" -v --timeout 300 \
    --timeout-method thread 2>&1 | grep -E "PASS|FAIL|passed|failed" | tail -40 ) > gpurun_out/r04o.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04o.txt | tail -50; exit $rc
