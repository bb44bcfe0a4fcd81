#!/bin/bash
# A/B of kernel build variants (same C-ABI): parity on the FK tests, then interleaved timing rounds.
#   bash tools/ab_xcd.sh <variant-suffix>...   (libkinhip<suffix>.so built by `make variant`)
set -u
mkdir -p gpurun_out
L=$PWD/kinematics.jl_amd/lib
VARS=("$@")
for v in "${VARS[@]}"; do
  KINHIP_LIB=$L/libkinhip$v.so timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "not ik" > gpurun_out/ab_test$v.log 2>&1
  rc=$?; echo "parity libkinhip$v rc=$rc: $(tail -n 1 gpurun_out/ab_test$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for r in 1 2 3; do
  for v in "${VARS[@]}"; do
    KINHIP_LIB=$L/libkinhip$v.so timeout -k 10 300 python tools/ab_probe.py 2> gpurun_out/ab_probe$v.err
    rc=$?; if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_probe$v.err; exit $rc; fi
  done
done
