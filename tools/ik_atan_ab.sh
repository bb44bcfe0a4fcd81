set -e
mkdir -p gpurun_out
for r in 1 2; do for v in 0 1; do for n in 65536 1048576; do
  KINHIP_IK_FAST_ATAN=$v AB_SPEC=1 AB_F32=1 IK_N=$n timeout -k 10 120 python tools/ik_ab.py >> gpurun_out/ikab_atan.txt 2>/dev/null
  echo "atan=$v n=$n done" >> gpurun_out/ikab_atan.txt
done; done; done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ik or nakamura" > gpurun_out/pytest_ik.log 2>&1
tail -3 gpurun_out/pytest_ik.log
cat gpurun_out/ikab_atan.txt
