#!/bin/bash
# Round 3: the GPU test suite (every step under its own time limit; stops at the first failure), then
# the fp32 collision error survey (tools/coll_fp32_err.py) for hardware and exact trig.
set -u
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r03_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/r03_gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/coll_fp32_err.py 20 > gpurun_out/r03_coll_err.txt 2>&1 || exit 1
timeout -k 10 300 env KINHIP_LIB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so KINHIP_COLL_FAST_TRIG=0 \
  python -u tools/coll_fp32_err.py 20 >> gpurun_out/r03_coll_err.txt 2>&1 || exit 1
cat gpurun_out/r03_coll_err.txt
