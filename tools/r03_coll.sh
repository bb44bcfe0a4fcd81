#!/bin/bash
# Round 3 collision kernel work: the collision GPU tests, then the config-5 legs of the bench (coll A/B driver)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_collision.py tests/test_gpu_coll_fp32_gate.py tests/test_random_trees.py \
  tests/test_gpu_parity.py -m gpu -x -q -k "coll or ineq or tree" --timeout 300 --timeout-method thread > gpurun_out/r03_coll_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_coll_tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED" gpurun_out/r03_coll_tests.log | head; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/r03_bench2.json 2> gpurun_out/r03_bench2.err || { tail gpurun_out/r03_bench2.err; exit 3; }
