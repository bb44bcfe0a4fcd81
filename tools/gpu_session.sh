#!/bin/bash
# One GPU session on the gpurun box: parity tests, smoke, bench, rocprof kernel trace.
# Stops at the first step that crashes or times out (exit codes other than 0/1).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name"; local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - t0 ))s)"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps 50 --warmup 10
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu
fi
