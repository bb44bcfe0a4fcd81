#!/bin/bash
# Round 3 IK analysis: dump the specialised IK source (A/B build, KINHIP_JIT_DUMP) and a rocprofv3 kernel
# trace + stats of the config-4 workload (tools/ik_ab.py, product library).
set -u
mkdir -p gpurun_out/jitdump gpurun_out/ikprof
export TMPDIR=/tmp
timeout -k 10 120 env KINHIP_LIB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so KINHIP_JIT_DUMP=$PWD/gpurun_out/jitdump/ik \
  AB_SPEC=1 AB_F32=1 IK_N=65536 python -u tools/ik_ab.py || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ikprof -o ik -- \
  python3 -u tools/ik_ab.py > gpurun_out/ikprof/run.log 2>&1 || exit 1
find gpurun_out/ikprof -name "*kernel_stats.csv" | head -3
for f in $(find gpurun_out/ikprof -name "*kernel_stats.csv"); do head -6 $f; done
