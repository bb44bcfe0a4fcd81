# round-4 session H: FK occupancy A/B (dynamic LDS caps on the specialised kernel) at 2^20 / 2^22 / 2^24 and
# in the Julia layout; then a JIT source dump of the f3 stage-2 kernel (ISA offline)
mkdir -p gpurun_out/jitdump
( FK_BIG=1 timeout -k 10 500 python -u tools/ab.py fk --reps 2 base KINHIP_FK_LDS=32768 KINHIP_FK_LDS=40960 \
    KINHIP_FK_LDS=53248 KINHIP_FK_LDS=65536 \
 && timeout -k 10 300 python -u tools/ab.py jl --reps 2 base KINHIP_FK_LDS=53248 KINHIP_FK_LDS=65536 \
 && KINHIP_LIB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so KINHIP_JIT_DUMP=$PWD/gpurun_out/jitdump \
    timeout -k 10 300 python -u tools/cik_bench.py 1024 ) > gpurun_out/r04h.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04h.txt | tail -30; ls gpurun_out/jitdump | head; exit $rc
