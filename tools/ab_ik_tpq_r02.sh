#!/bin/bash
# Two-phase IK (KINHIP_IK_TP_QUEUE bits: 1 = phase 1 on wave-local queues for large batches, 2 = phase 2
# on a grid bounded by the resident waves), batch sizes from the args (default 1M), two repetitions.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for tq in 0 1 2 3; do
    for n in ${@:-1048576}; do
      timeout -k 10 120 env KINHIP_IK_TP_QUEUE=$tq AB_SPEC=1 IK_N=$n python tools/ik_ab.py \
        2>/dev/null | sed "s/^/[tpq=$tq n=$n] /" || exit 1
    done
  done
done
