#!/bin/bash
# IK A/B: parity of each build on the IK tests, then timings per build x lanes-per-target.
set -u
mkdir -p gpurun_out
L=$PWD/kinematics.jl_amd/lib
for v in "" _w3 _w4; do
  KINHIP_LIB=$L/libkinhip$v.so timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "ik" > gpurun_out/ikab_test$v.log 2>&1
  rc=$?; echo "parity libkinhip$v rc=$rc: $(tail -n 1 gpurun_out/ikab_test$v.log)"
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/ikab_test$v.log; exit $rc; fi
done
for r in 1 2; do
  for v in "" _w3 _w4; do
    for g in 1 4; do
      KINHIP_IK_GROUP=$g KINHIP_LIB=$L/libkinhip$v.so timeout -k 10 300 python tools/ik_ab.py 2> gpurun_out/ikab$v.err || { tail -5 gpurun_out/ikab$v.err; exit 1; }
    done
  done
done
