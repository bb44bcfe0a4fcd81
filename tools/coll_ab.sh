#!/bin/bash
# k_coll A/B: collision parity tests per build, then interleaved timings.   bash tools/coll_ab.sh "" _u4 _u6
set -u
mkdir -p gpurun_out
L=$PWD/kinematics.jl_amd/lib
for v in "$@"; do
  KINHIP_LIB=$L/libkinhip$v.so timeout -k 10 600 python -m pytest tests/test_collision.py tests/test_planning.py -m gpu -x -q > gpurun_out/collab_test$v.log 2>&1
  rc=$?; echo "parity libkinhip$v rc=$rc: $(tail -n 1 gpurun_out/collab_test$v.log)"
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/collab_test$v.log; exit $rc; fi
done
for r in 1 2; do
  for v in "$@"; do
    KINHIP_LIB=$L/libkinhip$v.so timeout -k 10 300 python tools/coll_ab.py 2> gpurun_out/collab$v.err || { tail -5 gpurun_out/collab$v.err; exit 1; }
  done
done
