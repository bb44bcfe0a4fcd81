#!/bin/bash
# config-4 style IK at several batch sizes (product, specialised fp32), two rounds
set -u
for r in 1 2; do
for n in 65536 131072 262144 1048576; do
  timeout -k 10 120 env AB_SPEC=1 AB_F32=1 IK_N=$n python -u tools/ik_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/n=$n /" || exit 1
done
done
