# round-4 session Q: door sweep A/B, deferred scene gradient (new) vs the previous JIT sources (old)
set -o pipefail
mkdir -p gpurun_out
( for i in 1 2 3; do
    KINHIP_LIB=$PWD/kinematics.jl_amd/lib/libkinhip_oldjit.so timeout -k 10 200 python -u tools/scene_ab.py 15 | sed 's/^/old: /' || exit 1
    timeout -k 10 200 python -u tools/scene_ab.py 15 | sed 's/^/new: /' || exit 1
  done ) > gpurun_out/r04q.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04q.txt | tail -30; exit $rc
