#!/bin/bash
# k_coll A/B: occupancy hint for the gradient kernel and the AABB loop unroll (JIT knobs).
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "0 2" "6 2" "8 2" "0 1" "0 3" "0 6"; do
    set -- $cfg
    w=""; [ "$1" != 0 ] && w="KINHIP_JIT_COLL_WAVES=$1"
    timeout -k 10 120 env $w KINHIP_JIT_DEFS="-DKINHIP_AABB_UNROLL=$2" python tools/coll_spec_ab.py 2>/dev/null \
      | sed "s/^/waves=$1 unroll=$2 /" || exit 1
  done
done
