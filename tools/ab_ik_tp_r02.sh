#!/bin/bash
# Two-phase IK at 65k / 1M targets under compiler scheduling / occupancy options for the specialised
# kernels (KINHIP_JIT_OPTS raw options, KINHIP_JIT_IK_WAVES occupancy attribute), two repetitions.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "|" "-mllvm --amdgpu-sched-strategy=max-ilp|" "|1" "-mllvm --amdgpu-sched-strategy=max-ilp|1" "|2"; do
    o=${cfg%%|*}; w=${cfg##*|}
    for n in 65536 1048576; do
      timeout -k 10 120 env KINHIP_JIT_OPTS="$o" ${w:+KINHIP_JIT_IK_WAVES=$w} AB_SPEC=1 AB_F32=1 IK_N=$n python tools/ik_ab.py \
        2>/dev/null | sed "s/^/[opts=$o waves=$w] /" || exit 1
    done
  done
done
