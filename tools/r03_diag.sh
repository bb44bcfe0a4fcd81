#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/coll_spec_diff.py > gpurun_out/coll_spec_diff.txt 2>&1; cat gpurun_out/coll_spec_diff.txt | grep -v amdgpu.ids
bash tools/r03_ik_prof.sh
