# round-4 session B2: the tree collision-IK tests, smoke, the default bench, the layout probe, then the
# fault probe of the old generic 4-lane kernel (last: it may fault the GPU)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_collision_ik_tree.py -m gpu -v --timeout 300 \
    --timeout-method thread > gpurun_out/r04b2_tests.log 2>&1
rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/r04b2_tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04b_smoke.log 2>&1 \
  && tail -2 gpurun_out/r04b_smoke.log \
  && timeout -k 10 600 python -u bench.py > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err \
  && tail -c 600 gpurun_out/r04b_bench.json \
  && timeout -k 10 300 python -u tools/layout_probe.py > gpurun_out/r04b_layout.txt 2>&1 && cat gpurun_out/r04b_layout.txt \
  && bash tools/ikc_fault_session.sh
