#!/bin/bash
# A/B the kernel build variants (same C-ABI) on the GPU box: correctness of each
# variant on the parity tests, then interleaved bench rounds.
set -u
mkdir -p gpurun_out
L=kinematics.jl_amd/lib
for v in "" _bwd _nt _bwdnt; do
  echo "== parity libkinhip$v"
  KINHIP_LIB=$PWD/$L/libkinhip$v.so timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "not ik_dls_acceptance" > gpurun_out/ab_test$v.log 2>&1
  rc=$?; tail -n 2 gpurun_out/ab_test$v.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for r in 1 2; do
  for v in "" _bwd _nt _bwdnt; do
    KINHIP_LIB=$PWD/$L/libkinhip$v.so timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu > gpurun_out/ab_bench$v.$r.json 2> gpurun_out/ab_bench$v.$r.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench $v rc=$rc"; tail -5 gpurun_out/ab_bench$v.$r.err; exit $rc; fi
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_bench$v.$r.json')); print('$v'.ljust(8), 'r$r', '%.3e'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'us %.1f'%d['roofline']['avg_launch_us'], 'f64 %.3e'%d['fp64_fk_jac']['value'], 'cfg2 %.3e'%d['config2_fk6_f64']['value'])"
  done
done
timeout -k 10 120 python tools/bw_probe.py
