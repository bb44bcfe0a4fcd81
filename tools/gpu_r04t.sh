# round-4 session T: door-sweep compile-time variants through the tools build's JIT knobs
set -o pipefail
mkdir -p gpurun_out
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
( for v in base "-DKINHIP_AABB_UNROLL=1" "-DKINHIP_AABB_UNROLL=3" "-DKINHIP_AABB_UNROLL=6" "-DKINHIP_COLL_PAIRS=2" slp base; do
    if [ "$v" = base ]; then d=""; s=0; elif [ "$v" = slp ]; then d=""; s=1; else d="$v"; s=0; fi
    KINHIP_LIB=$AB KINHIP_JIT_DEFS="$d" KINHIP_JIT_SLP=$s timeout -k 10 200 python -u tools/scene_ab.py 15 | sed "s/^/$v: /" || exit 1
  done ) > gpurun_out/r04t.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04t.txt | tail -30; exit $rc
