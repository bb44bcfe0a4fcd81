#!/bin/bash
# Round evidence on the GPU box: gpu tests, smoke, bench (default args), rocprof trace+stats
# of the bench command, PMC passes of the headline kernel.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_session.sh test || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 3; }
cat gpurun_out/bench_default.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/bench -o bench -- python3 bench.py --no-cpu > gpurun_out/bench_rocprof.log 2>&1 || { tail gpurun_out/bench_rocprof.log; exit 4; }
tail -1 gpurun_out/bench_rocprof.log
for w in fkjac32ts fkjac64ts fk6_64ts ik32s coll32s collg32s; do bash tools/prof_session.sh $w || exit 5; done
timeout -k 10 600 python bench.py --no-cpu --sweep --steps 20 > gpurun_out/bench_sweep.json 2> gpurun_out/bench_sweep.err || { tail gpurun_out/bench_sweep.err; exit 9; }
