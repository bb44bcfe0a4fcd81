#!/bin/bash
# rocprofv3 passes for the round profiles: per workload a kernel trace + stats, then separate
# --pmc passes (never combined with trace domains; each pass within the per-block counter limits).
#   bash tools/pmc_passes.sh <tag>:<prof_kernel workload>[:extra args] ...
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
run() {  # run <dir> <args...>
  local d=$1; shift
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d gpurun_out/prof/$d -o $d -- python3 tools/prof_kernel.py $WARGS \
    > gpurun_out/prof_$d.log 2>&1
  local rc=$?; echo "$d rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof_$d.log; exit $rc; fi
}
for spec in "$@"; do
  IFS=: read -r TAG W EXTRA <<< "$spec"
  WARGS="--what $W --steps 20 $EXTRA"
  run ${TAG}_trace --kernel-trace --stats
  run ${TAG}_fetch --pmc FETCH_SIZE
  run ${TAG}_write --pmc WRITE_SIZE
  run ${TAG}_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
  run ${TAG}_sq2 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS
  case $TAG in fk*)
    run ${TAG}_mem --pmc TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE
    run ${TAG}_tlb --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum GRBM_GUI_ACTIVE ;;
  esac
done
