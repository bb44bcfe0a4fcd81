#!/bin/bash
# rocprofv3 passes on the GPU box: kernel trace + stats, then separate PMC passes
# (never combined with trace domains; MI355X_MICROARCH.md rocprofv3 section).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
W=${1:-fkjac32}
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 rocprofv3 "$@" --output-format csv -d gpurun_out/prof/$name -o $name -- python3 tools/prof_kernel.py --what $W --steps 20 > gpurun_out/prof_$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 gpurun_out/prof_$name.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
run ${W}_trace --kernel-trace --stats
run ${W}_fetch --pmc FETCH_SIZE
run ${W}_write --pmc WRITE_SIZE
run ${W}_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run ${W}_sq2 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
run ${W}_sq3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_WAVE_CYCLES
