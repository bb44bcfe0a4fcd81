set -u
mkdir -p gpurun_out
export KINHIP_JIT_DEFS="-DKINHIP_COLL_STPAIR=1"
timeout -k 10 300 python -u -m pytest tests/test_collision.py tests/test_planning.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/stpair_tests.log 2>&1 || { tail -30 gpurun_out/stpair_tests.log; exit 3; }
tail -2 gpurun_out/stpair_tests.log
for r in 1 2 3; do
  KINHIP_JIT_DEFS="" timeout -k 10 120 python tools/coll_spec_ab.py 2>/dev/null | sed 's/^/base  /' || exit 4
  KINHIP_JIT_DEFS="-DKINHIP_COLL_STPAIR=1" timeout -k 10 120 python tools/coll_spec_ab.py 2>/dev/null | sed 's/^/pair  /' || exit 5
done
