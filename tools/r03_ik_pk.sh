#!/bin/bash
# packed-FMA A/B (KINHIP_IK_PK) on the per-iteration probe, and a kernel trace of config 4 (specialised)
set -u
mkdir -p gpurun_out
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
for r in 1 2; do
for pk in 0 1; do
  timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_JIT_DEFS=-DKINHIP_IK_PK=$pk IK_NS=65536 python -u tools/ik_iter_probe.py 2>&1 \
    | grep -v amdgpu.ids | sed "s/^/pk=$pk /" || exit 1
  timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_JIT_DEFS=-DKINHIP_IK_PK=$pk AB_SPEC=1 AB_F32=1 python -u tools/ik_ab.py 2>&1 \
    | grep -v amdgpu.ids | sed "s/^/pk=$pk /" || exit 1
done
done
rm -rf gpurun_out/ikprof3; mkdir -p gpurun_out/ikprof3
timeout -k 10 300 env AB_SPEC=1 AB_F32=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ikprof3 -o ik -- \
  python3 -u tools/ik_ab.py > gpurun_out/ikprof3/run.log 2>&1 || exit 4
