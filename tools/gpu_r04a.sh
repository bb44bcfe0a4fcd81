# round-4 session A: the new collision-aware IK kernel (k_ik_tree) GPU tests, then the fault probe of the
# old generic 4-lane kernel (libkinhip_nocall.so / libkinhip_ab.so, built from the round-3 sources)
mkdir -p gpurun_out
T="timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$T tests/test_gpu_collision_ik.py tests/test_gpu_collision_ik_tree.py > gpurun_out/r04a_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r04a_tests.log | tail -40
[ $rc -ne 0 ] && exit $rc
bash tools/ikc_fault_session.sh
