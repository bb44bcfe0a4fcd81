#!/bin/bash
# k_coll A/B: store cache policy (KINHIP_STORE_AUX via KINHIP_JIT_DEFS) and the tile of the tiled layout.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_collision.py tests/test_planning.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for rep in 1 2; do
  for cfg in "2 8192" "0 8192" "2 4096" "0 4096" "2 16384"; do
    set -- $cfg
    timeout -k 10 120 env COLL_TILE=$2 KINHIP_JIT_DEFS="-DKINHIP_STORE_AUX=$1" python tools/coll_spec_ab.py 2>/dev/null \
      | sed "s/^/aux=$1 /" || exit 1
  done
done
