#!/bin/bash
# The one GPU-box session driver (replaces the per-round r0N_*.sh scripts).  Every GPU step runs under
# its own time limit and the script stops at the first failure; output goes under gpurun_out/.
#   gpurun -- bash tools/gpu_session.sh <step> [<step> ...]
# steps:
#   tests[=<pytest selection>]  the GPU suite (default: tests/), -x, per-test timeout
#   alltests=<pytest selection> the same without -x (every failure of a new batch of tests in one call)
#   isa                         the bench on the A/B build with KINHIP_JIT_CODE_DUMP (every specialised code object
#                               the bench compiles) + tools/isa_check.py over them and the generic kernels
#   smoke                       __graft_entry__.smoke()
#   bench                       python bench.py -> gpurun_out/bench.json
#   bench-driver                the driver's command (--gpus 1 --steps 20 --warmup 5) -> gpurun_out/bench_driver.json
#   bench-trace                 rocprofv3 --kernel-trace --stats of `bench.py --no-cpu` (gpurun_out/prof/bench)
#   sweep                       python bench.py --no-cpu --sweep -> gpurun_out/bench_sweep.json
#   rccl                        the RCCL test + the bench under a one-rank RCCL group (KINHIP_DIST_ALWAYS_GROUP=1)
#   pmc=<tag>:<workload>[,...]  per workload a kernel trace + stats, then separate --pmc passes (never with
#                               trace domains; each pass within the per-block counter limits); workloads of
#                               tools/prof_kernel.py (e.g. fkjac32ts, ik32s, coll32s, collg32s, cik32s)
#   ik                          config-4 IK timing (product, twice) and 1M targets; per-iteration probe
#   ik-sections                 iteration section stamps (A/B build, -DKINHIP_IK_SECT=k)
#   ikt-sections[=<defs>]       collision-aware IK (f3 stage 2) section stamps (A/B build, -DKINHIP_IKT_SECT=k
#                               plus the given definitions, e.g. ikt-sections=-DKINHIP_IKT_OWN=0)
#   ik-timeline                 per-lane entry / write timeline of one solve (A/B build)
#   ik-dump                     the specialised IK source (A/B build, KINHIP_JIT_DUMP) + a kernel trace of config 4
#   coll                        the plain-row padding A/B of the config-5 legs (tools/coll_pad_ab.py)
#   cik                         the f3 bistage IK leg split by stage, stage 2 on one lane vs 4 (tools/cik_bench.py)
#   dumps                       the specialised IK (fp32 + fp64) and collision-IK sources (A/B build, KINHIP_JIT_DUMP)
#   coll-dump                   the specialised collision source (A/B build, KINHIP_JIT_DUMP) for offline ISA
#   ab=<workload>:<setting>[;<setting>...]   tools/ab.py (A/B build), e.g. ab=ik:base;KINHIP_IK_P2_WAVES=4
#   pr2-miss[=<n>]              tools/pr2_miss_study.py (PR2 collision-IK leg misses vs host SLSQP)
#   pr2-alt                     tools/pr2_alt_probe.py (stage-2 step budgets from the manip pose, alt schedules)
#   scene-const                 door sweep A/B: scene tables as data vs compiled in (tools/scene_ab.py), x3 each,
#                               plus a rocprofv3 kernel trace of both (VGPR counts)
#   pts-probe                   tools/pts_probe (hipStreamPerThread after thread exit vs hipDeviceSynchronize)
#   srcab=<tool.py>:<reps>      the A/B build's specialised kernels from the device headers of gpurun_ab/old (fill it
#                               first: git show <rev>:kinematics.jl_amd/csrc/<h> > gpurun_ab/old/<h> for the six
#                               kinhip_{prog,device,fk_dev,ik_dev,coll_dev,ikt_dev}.h) vs csrc/ (KINHIP_JIT_SRC_DIR),
#                               alternated <reps> times; any KINHIP_JIT_SRC_DIR in the caller's environment also
#                               applies to the other steps (e.g. ikt-sections)
set -u -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
AB=$PWD/kinematics.jl_amd/lib/libkinhip_ab.so
quiet() { grep -v "amdgpu.ids" || true; }

pmc_run() {  # pmc_run <dir> <workload args> <rocprofv3 args...>
  local d=$1 w=$2; shift 2
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d gpurun_out/prof/$d -o $d -- python3 tools/prof_kernel.py $w \
    > gpurun_out/prof_$d.log 2>&1
  local rc=$?; echo "$d rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$d.log; exit $rc; }
}

for step in "$@"; do
  echo "== $step"
  case $step in
    tests|tests=*)
      sel=${step#tests}; sel=${sel#=}; sel=${sel:-tests}
      timeout -k 10 1500 python -u -m pytest $sel -m gpu -x -v --timeout 300 --timeout-method thread \
        > gpurun_out/gpu_tests.log 2>&1
      rc=$?; tail -3 gpurun_out/gpu_tests.log
      [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -30; exit $rc; } ;;
    alltests=*)
      sel=${step#alltests=}
      timeout -k 10 1500 python -u -m pytest $sel -m gpu -v --timeout 300 --timeout-method thread \
        > gpurun_out/gpu_tests_all.log 2>&1
      rc=$?; tail -3 gpurun_out/gpu_tests_all.log
      [ $rc -eq 0 ] || grep -E "FAILED|Error" gpurun_out/gpu_tests_all.log | head -30 ;;
    isa)
      mkdir -p gpurun_out/isa
      timeout -k 10 400 env KINHIP_LIB=$AB KINHIP_JIT_CODE_DUMP=$PWD/gpurun_out/isa/jit KINHIP_JIT_DUMP=$PWD/gpurun_out/isa/src \
        python bench.py --no-cpu > gpurun_out/isa/bench_ab.json 2> gpurun_out/isa/bench_ab.err || { tail gpurun_out/isa/bench_ab.err; exit 9; }
      python tools/isa_check.py gpurun_out/isa/jit.*.co > gpurun_out/isa/isa_check.txt 2>&1; tail -3 gpurun_out/isa/isa_check.txt ;;
    pr2-alt)
      timeout -k 10 600 python tools/pr2_alt_probe.py > gpurun_out/pr2_alt_probe.json 2> gpurun_out/pr2_alt_probe.err \
        || { tail -20 gpurun_out/pr2_alt_probe.err; exit 12; }
      cat gpurun_out/pr2_alt_probe.json ;;
    pr2-miss|pr2-miss=*)
      n=${step#pr2-miss}; n=${n#=}; n=${n:-200}
      timeout -k 10 900 python tools/pr2_miss_study.py $n > gpurun_out/pr2_miss_study.json 2> gpurun_out/pr2_miss_study.err \
        || { tail -20 gpurun_out/pr2_miss_study.err; exit 11; }
      cut -c1-1500 gpurun_out/pr2_miss_study.json ;;
    scene-const)
      for r in 1 2 3; do
        for c in 0 1; do
          timeout -k 10 120 env SCENE_AB_CONST=$c python tools/scene_ab.py 15 2>&1 | quiet || exit 12
        done
      done
      for c in 0 1; do
        timeout -k 10 180 env SCENE_AB_CONST=$c rocprofv3 --kernel-trace --stats --output-format csv \
          -d gpurun_out/prof/scene$c -o scene$c -- python3 tools/scene_ab.py 3 > gpurun_out/prof_scene$c.log 2>&1 \
          || { tail -5 gpurun_out/prof_scene$c.log; exit 12; }
      done ;;
    pts-probe)
      timeout -k 10 60 tools/pts_probe > gpurun_out/pts_probe.txt 2>&1; rc=$?; cat gpurun_out/pts_probe.txt
      [ $rc -eq 0 ] || exit 10 ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | quiet || exit 2 ;;
    bench)
      timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 3; }
      cut -c1-400 gpurun_out/bench.json ;;
    bench-driver)
      timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json \
        2> gpurun_out/bench_driver.err || { tail gpurun_out/bench_driver.err; exit 3; }
      cut -c1-300 gpurun_out/bench_driver.json ;;
    bench-trace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/bench -o bench -- \
        python3 bench.py --no-cpu > gpurun_out/bench_rocprof.log 2>&1 || { tail gpurun_out/bench_rocprof.log; exit 4; } ;;
    sweep)
      timeout -k 10 600 python bench.py --no-cpu --sweep --steps 20 > gpurun_out/bench_sweep.json \
        2> gpurun_out/bench_sweep.err || { tail gpurun_out/bench_sweep.err; exit 5; } ;;
    rccl)
      timeout -k 10 240 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
        > gpurun_out/rccl_tests.log 2>&1 || { tail -20 gpurun_out/rccl_tests.log; exit 6; }
      tail -2 gpurun_out/rccl_tests.log
      timeout -k 10 400 env KINHIP_DIST_ALWAYS_GROUP=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --no-cpu > gpurun_out/bench_rccl_1rank.json \
        2> gpurun_out/bench_rccl_1rank.err || { tail gpurun_out/bench_rccl_1rank.err; exit 6; } ;;
    pmc=*)
      IFS=, read -ra specs <<< "${step#pmc=}"
      for spec in "${specs[@]}"; do
        IFS=: read -r TAG W EXTRA <<< "$spec"
        WARGS="--what $W --steps 20 ${EXTRA:-}"
        pmc_run ${TAG}_trace "$WARGS" --kernel-trace --stats
        pmc_run ${TAG}_fetch "$WARGS" --pmc FETCH_SIZE
        pmc_run ${TAG}_write "$WARGS" --pmc WRITE_SIZE
        pmc_run ${TAG}_sq "$WARGS" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
        pmc_run ${TAG}_sq2 "$WARGS" --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY \
          SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS
        case $TAG in fk*)
          pmc_run ${TAG}_mem "$WARGS" --pmc TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE
          pmc_run ${TAG}_tlb "$WARGS" --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
            TCP_UTCL1_REQUEST_sum GRBM_GUI_ACTIVE ;;
        esac
      done ;;
    ik)
      for r in 1 2; do timeout -k 10 120 env AB_SPEC=1 IK_N=65536 python -u tools/ik_ab.py 2>&1 | quiet || exit 8; done
      timeout -k 10 120 env AB_SPEC=1 IK_N=1048576 AB_F32=1 python -u tools/ik_ab.py 2>&1 | quiet || exit 8
      timeout -k 10 200 python -u tools/ik_iter_probe.py 2>&1 | quiet || exit 8 ;;
    ik-sections)
      for k in 1 2 3 4 5 6 7; do
        timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=$k python -u tools/ik_sect.py 2>&1 | quiet || exit 8
      done ;;
    ikt-sections|ikt-sections=*)
      xd=${step#ikt-sections}; xd=${xd#=}
      for k in 1 2 3 4 5 6 7; do
        timeout -k 10 180 env KINHIP_LIB=$AB "KINHIP_JIT_DEFS=-DKINHIP_IKT_SECT=$k $xd" python -u tools/ikt_sect.py 2>&1 | quiet || exit 8
      done ;;
    ik-timeline)
      timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=9 python -u tools/ik_timeline.py 2>&1 | quiet || exit 8 ;;
    ik-dump)
      mkdir -p gpurun_out/jit gpurun_out/ikprof
      timeout -k 10 120 env KINHIP_LIB=$AB KINHIP_JIT_DUMP=$PWD/gpurun_out/jit/ik AB_SPEC=1 AB_F32=1 IK_N=65536 \
        python -u tools/ik_ab.py 2>&1 | quiet || exit 8
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ikprof -o ik -- python3 -u tools/ik_ab.py \
        > gpurun_out/ikprof/run.log 2>&1 || exit 7 ;;
    dumps)  # the specialised IK sources (both precisions) and the collision-IK ones, for offline ISA work
      mkdir -p gpurun_out/jit
      timeout -k 10 200 env KINHIP_LIB=$AB KINHIP_JIT_DUMP=$PWD/gpurun_out/jit/ik AB_SPEC=1 IK_N=65536 \
        python -u tools/ik_ab.py 2>&1 | quiet || exit 8
      timeout -k 10 300 env KINHIP_LIB=$AB KINHIP_JIT_DUMP=$PWD/gpurun_out/jit/cik AB_SPEC=1 \
        python -u tools/cik_ab.py 2>&1 | quiet || exit 8 ;;
    coll)
      timeout -k 10 200 python -u tools/coll_pad_ab.py 2>&1 | quiet || exit 8 ;;
    cik)
      timeout -k 10 200 python -u tools/cik_bench.py 2>&1 | quiet || exit 8 ;;
    coll-dump)
      mkdir -p gpurun_out/jit
      timeout -k 10 200 env KINHIP_LIB=$AB KINHIP_JIT_DUMP=$PWD/gpurun_out/jit/coll AB_SPEC=1 \
        python -u tools/coll_spec_ab.py 2>&1 | quiet || exit 8 ;;
    srcab=*)  # srcab=<tool.py>:<reps>: the A/B build with the JIT device headers of gpurun_ab/old vs csrc/, alternated
      spec=${step#srcab=}; tool=${spec%%:*}; reps=${spec#*:}
      for r in $(seq 1 $reps); do
        for d in gpurun_ab/old kinematics.jl_amd/csrc; do
          echo "[$d]"
          timeout -k 10 300 env KINHIP_LIB=$AB KINHIP_JIT_SRC_DIR=$PWD/$d python -u tools/$tool 2>&1 | quiet || exit 8
        done
      done ;;
    ab=*)
      spec=${step#ab=}; w=${spec%%:*}; IFS=';' read -ra sets <<< "${spec#*:}"
      timeout -k 10 900 python -u tools/ab.py $w "${sets[@]}" 2>&1 | quiet || exit 8 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
