# round-4 session R: the whole GPU suite, smoke, the default bench and its rocprofv3 kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=15 --timeout 300 --timeout-method thread \
    > gpurun_out/r04r_tests.log 2>&1
rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/r04r_tests.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04r_smoke.log 2>&1 \
  && tail -2 gpurun_out/r04r_smoke.log \
  && timeout -k 10 600 python -u bench.py > gpurun_out/r04r_bench.json 2> gpurun_out/r04r_bench.err \
  && tail -c 300 gpurun_out/r04r_bench.json \
  && timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/bench -o bench -- \
     python3 bench.py --no-cpu > gpurun_out/r04r_bench_rocprof.log 2>&1 \
  && ls gpurun_out/prof/bench
