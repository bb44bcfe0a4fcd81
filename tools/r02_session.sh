#!/bin/bash
# Round-2 GPU session steps (run on the gpurun box from the repo root):
#   bash tools/r02_session.sh <step>...
# Steps: iktest ikab probe trace bench pytest smoke.  Every GPU step has its own time limit; the
# script stops at the first step that fails.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/kinematics.jl_amd/lib
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name"; local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - t0 ))s)"; tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    iktest) step iktest 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "ik_dls" ;;
    ikab)
      for n in 65536 1048576; do
        for qm in 0 1 2; do
          step ikab_${n}_q$qm 300 env AB_SPEC=1 AB_F32=1 IK_N=$n KINHIP_IK_QUEUE=$qm python tools/ik_ab.py
        done
      done ;;
    probe) step tile_probe126 300 $L/tile_probe 126 ;;
    trace) step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/bench -o bench -- python3 bench.py --steps 50 --warmup 10 --no-cpu ;;
    bench) step bench 900 python bench.py --steps 50 --warmup 10 ;;
    pytest) step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    dist2) step dist2 600 env KINHIP_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
             --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
