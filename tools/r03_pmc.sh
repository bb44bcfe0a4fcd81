#!/bin/bash
# Round 3 PMC passes (tools/pmc_passes.sh): IK config 4, collision min / dists+grads plain / tiled, FK headline
set -u
rm -rf gpurun_out/prof
bash tools/pmc_passes.sh ik32s:ik32s coll32s:coll32s collg32s:collg32s collg32ts:collg32ts fkjac32ts:fkjac32ts
