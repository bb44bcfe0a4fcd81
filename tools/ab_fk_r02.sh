#!/bin/bash
# FK grid-strided variant: parity (the large-batch test runs the strided kernel), then timings with
# KINHIP_FK_PER_LANE forced to 1 / 2 / 3 and the automatic choice.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32_gate.py -x -q \
  --timeout 300 --timeout-method thread -k "fk or golden or ground or specialized or gate" > gpurun_out/ab_fk_tests.log 2>&1 \
  || { tail -30 gpurun_out/ab_fk_tests.log; exit 1; }
tail -1 gpurun_out/ab_fk_tests.log
for rep in 1 2; do
  for k in 1 2 3 auto; do
    if [ $k = auto ]; then
      timeout -k 10 120 python tools/fk_stride_ab.py 2>/dev/null || exit 1
    else
      timeout -k 10 120 env KINHIP_FK_PER_LANE=$k python tools/fk_stride_ab.py 2>/dev/null || exit 1
    fi
  done
done
