#!/bin/bash
# IK two-phase schedule at 32k / 65k / 1M (KINHIP_IK_TWO_PHASE: unset = automatic, 0 = off, 1 = forced).
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for v in auto 0 1; do
    for n in 32768 65536 1048576; do
      if [ $v = auto ]; then e=""; else e="KINHIP_IK_TWO_PHASE=$v"; fi
      timeout -k 10 120 env $e AB_SPEC=1 IK_N=$n python tools/ik_ab.py 2>/dev/null | sed "s/^/two=$v n=$n /" || exit 1
    done
  done
done
