# round-4 session F: config-4 IK iteration sections (A/B build stamps) with the fp64 and the fp32 solve, then
# the profiling session C (bench trace + PMC passes)
mkdir -p gpurun_out
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
for f in 1 0; do
  for k in 1 2 3 4 5 6 7; do
    timeout -k 10 120 env KINHIP_LIB=$AB "KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=$k -DKINHIP_IK_F64SOLVE=$f" \
      python -u tools/ik_sect.py 2>&1 | grep -v amdgpu.ids | sed "s/^/f64solve=$f /" || exit 8
  done
done > gpurun_out/r04f_ik_sections.txt
cat gpurun_out/r04f_ik_sections.txt
bash tools/gpu_r04c.sh
