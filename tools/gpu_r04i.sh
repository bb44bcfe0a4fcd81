# round-4 session I: collision-kernel occupancy A/B (config 5 legs and the door sweep), then the bench with
# the FK occupancy cap
mkdir -p gpurun_out
( timeout -k 10 500 python -u tools/ab.py coll --reps 2 base KINHIP_COLL_LDS=32768 KINHIP_COLL_LDS=53248 \
    KINHIP_COLL_LDS=65536 \
 && timeout -k 10 600 python -u bench.py > gpurun_out/r04i_bench.json 2> gpurun_out/r04i_bench.err ) \
  > gpurun_out/r04i.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04i.txt; tail -c 300 gpurun_out/r04i_bench.json; exit $rc
