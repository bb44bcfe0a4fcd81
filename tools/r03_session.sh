#!/bin/bash
# Round 3 evidence, call 1: the GPU test suite, smoke(), the default bench line and a rocprofv3
# kernel trace + stats of the same bench command (every GPU step under its own limit; stops at the
# first failure).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/r03_gpu_tests.log | head -30; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 2
timeout -k 10 400 python bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { tail gpurun_out/r03_bench.err; exit 3; }
cat gpurun_out/r03_bench.json
mkdir -p gpurun_out/ikprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ikprof -o ik -- python3 -u tools/ik_ab.py \
  > gpurun_out/ikprof/run.log 2>&1 || exit 4
for f in $(find gpurun_out/ikprof -name "*kernel_stats.csv"); do head -8 $f | cut -c1-200; done
