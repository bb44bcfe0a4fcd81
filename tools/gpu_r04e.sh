# round-4 session E: kernel traces of config-4 IK (phase 1 / phase 2 durations) for the round-3 settings and
# the damped ones, then the tree collision-IK tests and the f3 legs after the DPP row broadcast
mkdir -p gpurun_out/prof
export TMPDIR=/tmp AB_F32=1 AB_SPEC=1 KINHIP_LIB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/ikA -o ikA -- \
    python3 tools/ik_ab.py > gpurun_out/r04e_ikA.log 2>&1 \
 && IK_DAMP=0.01 IK_MAXSTEP=1.0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/prof/ikB -o ikB -- python3 tools/ik_ab.py > gpurun_out/r04e_ikB.log 2>&1 \
 && unset KINHIP_LIB AB_F32 AB_SPEC \
 && timeout -k 10 600 python -u -m pytest tests/test_gpu_collision_ik_tree.py tests/test_gpu_collision_ik.py -m gpu -v \
    --timeout 300 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1 \
 && timeout -k 10 300 python -u tools/cik_bench.py > gpurun_out/r04e_cik.txt 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r04e_tests.log | tail -3
grep -v amdgpu.ids gpurun_out/r04e_cik.txt | tail -12
for f in gpurun_out/prof/ikA/ikA_kernel_stats.csv gpurun_out/prof/ikB/ikB_kernel_stats.csv; do
  [ -f $f ] && grep -E "ik_6|Name" $f | cut -d, -f1-5
done
exit $rc
