# round-4 session N: config-4 per-lane timelines (fixed / damped), then the whole GPU suite, smoke and the bench
mkdir -p gpurun_out
bash tools/gpu_r04m.sh; true
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=15 --timeout 300 --timeout-method thread \
    > gpurun_out/r04n_tests.log 2>&1
rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/r04n_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04n_smoke.log 2>&1 \
  && tail -2 gpurun_out/r04n_smoke.log \
  && timeout -k 10 600 python -u bench.py > gpurun_out/r04n_bench.json 2> gpurun_out/r04n_bench.err \
  && tail -c 300 gpurun_out/r04n_bench.json
