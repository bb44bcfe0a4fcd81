#!/bin/bash
# Scheduler-strategy A/B for the specialised kernels (KINHIP_JIT_OPTS passes raw options to hiprtc).
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for o in "" "-mllvm --amdgpu-sched-strategy=max-ilp" "-mllvm --amdgpu-schedule-metric-bias=0"; do
    timeout -k 10 120 env KINHIP_JIT_OPTS="$o" AB_SPEC=1 AB_F32=1 IK_N=65536 python tools/ik_ab.py 2>/dev/null | sed "s/^/[$o] /" || exit 1
    timeout -k 10 120 env KINHIP_JIT_OPTS="$o" AB_SPEC=1 AB_F32=1 IK_N=1048576 python tools/ik_ab.py 2>/dev/null | sed "s/^/[$o] /" || exit 1
    timeout -k 10 120 env KINHIP_JIT_OPTS="$o" python tools/coll_spec_ab.py 2>/dev/null | sed "s/^/[$o] /" || exit 1
    timeout -k 10 120 env KINHIP_JIT_OPTS="$o" python tools/fk_legs_ab.py 2>/dev/null | sed "s/^/[$o] /" || exit 1
  done
done
