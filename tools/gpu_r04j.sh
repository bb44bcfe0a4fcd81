# round-4 session J: FK workgroup size x LDS cap A/B (the specialised kernel) and the probe's sweep over the
# same occupancies
mkdir -p gpurun_out
( FK_BIG=1 timeout -k 10 500 python -u tools/ab.py fk --reps 2 base KINHIP_FK_BLOCK=128 \
    KINHIP_FK_BLOCK=128,KINHIP_FK_LDS=53248 KINHIP_FK_BLOCK=64,KINHIP_FK_LDS=16384 \
 && timeout -k 10 300 python -u tools/ab.py jl --reps 2 base KINHIP_FK_BLOCK=128 \
 && timeout -k 10 300 python -u tools/probe_occ.py ) > gpurun_out/r04j.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04j.txt; exit $rc
