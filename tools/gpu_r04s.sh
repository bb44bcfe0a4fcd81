# round-4 session S: keep the generated JIT sources of the door-sweep plan (KINHIP_JIT_DUMP, tools build)
set -o pipefail
mkdir -p gpurun_out/jit
KINHIP_LIB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so KINHIP_JIT_DUMP=$PWD/gpurun_out/jit/coll \
  timeout -k 10 200 python -u tools/scene_ab.py 3 && ls -la gpurun_out/jit
