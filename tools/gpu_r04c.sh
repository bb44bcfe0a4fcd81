# round-4 session C: rocprofv3 kernel trace + stats of the bench, then the PMC passes of the headline
# (tiled), the Julia layout (plain rows, ld = N), config-4 IK, the door sweep and the collision IK stage 2
# (f3 and the pillar scene); tags are tools/summarize_prof.py's workload names
bash tools/gpu_session.sh bench-trace \
  "pmc=fkjac32ts:fkjac32ts,fkjac32sjl:fkjac32s:--pad 0,ik32s:ik32s,scene32s:scene32s,cik32s:cik32s,cikp32s:cikp32s"
