#!/bin/bash
# Round-2 A/B on one box: collision parity + timings of the specialised k_coll legs, IK occupancy /
# lane-group settings, and the list of PMC counters this rocprofv3 offers.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_collision.py tests/test_planning.py tests/test_gpu_collision_ik.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for rep in 1 2; do
  timeout -k 10 120 python tools/coll_spec_ab.py 2>/dev/null || exit 1
  for cfg in "4 0" "4 4" "2 0" "8 0"; do
    set -- $cfg
    if [ "$2" = 0 ]; then
      timeout -k 10 120 env AB_SPEC=1 AB_F32=1 IK_N=65536 KINHIP_IK_GROUP=$1 python tools/ik_ab.py 2>/dev/null | sed "s/^/waves=auto /" || exit 1
    else
      timeout -k 10 120 env AB_SPEC=1 AB_F32=1 IK_N=65536 KINHIP_IK_GROUP=$1 KINHIP_JIT_IK_WAVES=$2 python tools/ik_ab.py 2>/dev/null | sed "s/^/waves=$2 /" || exit 1
    fi
  done
done
timeout -k 10 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
grep -c . gpurun_out/rocprof_counters.txt
