#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -n 3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
KINHIP_NO_WIDE=1 timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -k "golden or vs_oracle or edge or large" > gpurun_out/pytest_gpu_narrow.log 2>&1; rc=$?; tail -n 2 gpurun_out/pytest_gpu_narrow.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2 3; do
  for v in wide narrow; do
    if [ $v = narrow ]; then export KINHIP_NO_WIDE=1; else unset KINHIP_NO_WIDE; fi
    timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu > gpurun_out/abw_$v.$r.json 2> gpurun_out/abw_$v.$r.err || { tail -5 gpurun_out/abw_$v.$r.err; exit 3; }
    python -c "import json; d=json.load(open('gpurun_out/abw_$v.$r.json')); print('$v'.ljust(7), 'r$r', '%.3e'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'us %.1f'%d['roofline']['avg_launch_us'], 'f64 %.3e (%.1f us)'%(d['fp64_fk_jac']['value'], d['fp64_fk_jac']['avg_launch_us']), 'cfg2 %.3e (%.1f us)'%(d['config2_fk6_f64']['value'], d['config2_fk6_f64']['avg_launch_us']))"
  done
done
