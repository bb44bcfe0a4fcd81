#!/bin/bash
# Round 3: the GPU test suite (every step under its own time limit; stops at the first failure), the
# fp32 collision error survey (tools/coll_fp32_err.py) for hardware and exact trig, config-4 IK
# timings and a rocprofv3 kernel trace of the IK leg.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r03_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r03_gpu_tests.log | head -30; exit $rc; }
for k in 1 2; do
  timeout -k 10 120 env AB_SPEC=1 IK_N=65536 python -u tools/ik_ab.py || exit 1
  timeout -k 10 120 env AB_SPEC=1 IK_N=1048576 AB_F32=1 python -u tools/ik_ab.py || exit 1
done
timeout -k 10 300 python -u tools/coll_fp32_err.py 20 > gpurun_out/r03_coll_err.txt 2>&1 || exit 1
timeout -k 10 300 env KINHIP_LIB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so KINHIP_COLL_FAST_TRIG=0 \
  python -u tools/coll_fp32_err.py 20 >> gpurun_out/r03_coll_err.txt 2>&1 || exit 1
cat gpurun_out/r03_coll_err.txt
