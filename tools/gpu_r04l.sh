# round-4 session L: LDS-staged FK row stores (A/B build) in the headline / big-batch / Julia layouts, the probe
# sweep with the staged-store pattern, and the collision legs again (door sweep variance)
mkdir -p gpurun_out
( FK_BIG=1 timeout -k 10 500 python -u tools/ab.py fk --reps 2 base \
    "KINHIP_JIT_DEFS=-DKINHIP_FK_STAGE=1,KINHIP_FK_STAGE_ON=1" \
 && timeout -k 10 300 python -u tools/ab.py jl --reps 2 base "KINHIP_JIT_DEFS=-DKINHIP_FK_STAGE=1,KINHIP_FK_STAGE_ON=1" \
 && timeout -k 10 300 python -u tools/probe_occ.py \
 && timeout -k 10 300 python -u tools/ab.py coll --reps 2 base ) > gpurun_out/r04l.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04l.txt; exit $rc
