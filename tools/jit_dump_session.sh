set -u
mkdir -p gpurun_out/jit gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 120 env KINHIP_JIT_DUMP=gpurun_out/jit/ik AB_SPEC=1 AB_F32=1 python tools/ik_ab.py || exit 1
timeout -k 10 120 env KINHIP_JIT_DUMP=gpurun_out/jit/coll python tools/coll_spec_ab.py || exit 1
timeout -k 10 200 env KINHIP_JIT_IK_WAVES=4 AB_SPEC=1 AB_F32=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/ikw4 -o ikw4 -- python3 tools/ik_ab.py || exit 1
ls gpurun_out/jit
