#!/bin/bash
# A/B of the specialised fp32 IK kernel's occupancy request (KINHIP_JIT_IK_WAVES, unset = compiler's
# choice) at 65k and 1M targets, interleaved, two rounds.
set -e
mkdir -p gpurun_out
for r in 1 2; do for v in 0 4; do for n in 65536 1048576; do
  KINHIP_JIT_IK_WAVES=$v AB_SPEC=1 AB_F32=1 IK_N=$n timeout -k 10 120 python tools/ik_ab.py >> gpurun_out/ikab_waves.txt 2>/dev/null
  echo "waves=$v n=$n" >> gpurun_out/ikab_waves.txt
done; done; done
cat gpurun_out/ikab_waves.txt
