# round-4 session P: the scene union's gradient deferred to the winning group (door sweep A/B against the
# previous JIT sources, alternating libraries in one box), then the scene / tree collision tests
set -o pipefail
mkdir -p gpurun_out
( for i in 1 2; do
    KINHIP_LIB=$PWD/kinematics.jl_amd/lib/libkinhip_oldjit.so timeout -k 10 200 python -u tools/coll_spec_ab.py | sed 's/^/old: /' || exit 1
    timeout -k 10 200 python -u tools/coll_spec_ab.py | sed 's/^/new: /' || exit 1
  done
  timeout -k 10 900 python -u -m pytest tests/test_collision.py tests/test_gpu_collision_ik_tree.py tests/test_gpu_collision_ik.py \
    -m gpu -x -v --timeout 300 --timeout-method thread 2>&1 | grep -E "PASS|FAIL|ERROR|passed|failed|Error" | tail -80 ) > gpurun_out/r04p.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04p.txt | tail -90; exit $rc
