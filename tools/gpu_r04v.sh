# round-4 session V: half-attempt phase-1 cut for damped IK -- the IK GPU tests, smoke and the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ik_fp32_bound.py tests/test_gpu_ik_rpy.py -m gpu -k "ik" \
    -v --timeout 300 --timeout-method thread > gpurun_out/r04v_tests.log 2>&1
rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/r04v_tests.log | tail -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04v_smoke.log 2>&1 \
  && tail -1 gpurun_out/r04v_smoke.log \
  && timeout -k 10 600 python -u bench.py > gpurun_out/r04v_bench.json 2> gpurun_out/r04v_bench.err \
  && tail -c 200 gpurun_out/r04v_bench.json
