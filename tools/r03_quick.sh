#!/bin/bash
# Round 3: a subset of the GPU tests (args = pytest selection), each run under a time limit.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r03_quick.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|batched|passed|failed" gpurun_out/r03_quick.log | tail -40
exit $rc
