"""Two host threads on hipStreamPerThread: the handle ((hipStream_t)2) names each calling
thread's own default stream, so the two-phase IK's "same stream as last time" shortcut must not hand one
thread's in-flight scratch set (hand-over rings, fail lists) to the other.  Both threads run config-4 sized
batches (two-phase schedule) back to back on that handle, each into its own outputs; every result must
equal the single-threaded reference bit for bit.  The same with one explicit stream per thread, and with
one thread on the per-thread handle, as controls."""
import ctypes as C
import os
import threading

import pytest
import torch

from conftest import ARM, golden

import kinhip
from kinhip import _lib as K

pytestmark = pytest.mark.gpu

HIP_STREAM_PER_THREAD = 2


@pytest.fixture(scope="module")
def config4():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dev = torch.device("cuda", 0)
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32).specialize()
    N = 65536  # more than one round of waves: the two-phase schedule and its scratch sets
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, seed=31,
                                dtype=torch.float32, device=dev)
    tgt = plan.run(Qt)[0][0].contiguous()
    Q0 = torch.zeros((8, N), dtype=torch.float32, device=dev)
    kw = dict(max_iters=64, restarts=3, seed=0, lam=1e-2, max_step=0.5, tol_pos=1e-3, tol_rot=1e-3)
    ref_q, ref_it, _ = plan.ik_dls(tgt, torch.empty_like(Q0), Q0=Q0, **kw)
    torch.cuda.synchronize()
    return dev, plan, tgt, Q0, ref_q, ref_it, N


def _hip():
    return C.CDLL("libamdhip64.so.7")  # (the runtime torch has loaded: same soname, same instance)


def _run(config4, n_threads, streams, reps=6, sync_in_thread=True):
    dev, plan, tgt, Q0, ref_q, ref_it, N = config4
    prm = K.IkParams(64, 1e-2, 1e-3, 1e-3, 0.5, 1, 3, 0, 0, 0, 0.0)
    outs = [[(torch.empty_like(Q0), torch.empty(N, dtype=torch.int32, device=dev)) for _ in range(reps)]
            for _ in range(n_threads)]
    errors = []
    barrier = threading.Barrier(n_threads)

    def worker(t):
        try:
            torch.cuda.set_device(dev)
            st = C.c_void_p(streams[t])
            barrier.wait()
            for Q, it in outs[t]:
                K.check(K.lib().kin_ik_dls_batch_from(plan._h, C.byref(prm), tgt.data_ptr(), N, Q0.data_ptr(),
                                                      Q.data_ptr(), N, N, it.data_ptr(), None, N, st))
            # a thread's per-thread default stream is its own: the thread waits for it before it ends (the
            # device-wide synchronize below does not cover the streams of threads that have exited)
            if sync_in_thread:
                assert _hip().hipStreamSynchronize(st) == 0
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    torch.cuda.synchronize()
    assert not errors, errors
    bad = [[int((it != ref_it).sum()) + int((Q != ref_q).any(0).sum()) for Q, it in outs[t]] for t in range(n_threads)]
    return bad


def test_two_threads_on_the_per_thread_stream_handle(config4, reps=int(os.environ.get("STREAMS_REPS", "6"))):
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    controls = {"one thread, per-thread handle": _run(config4, 1, [HIP_STREAM_PER_THREAD], reps),
                "two threads, own streams": _run(config4, 2, [s1.cuda_stream, s2.cuda_stream], reps)}
    got = _run(config4, 2, [HIP_STREAM_PER_THREAD, HIP_STREAM_PER_THREAD], reps)
    # (diagnostic, not asserted: without the in-thread synchronize, whether the device-wide one after
    # the threads have ended covers their per-thread streams)
    nosync = _run(config4, 2, [HIP_STREAM_PER_THREAD, HIP_STREAM_PER_THREAD], reps, sync_in_thread=False)
    print("mismatching targets per call:", controls, "two threads, per-thread handle:", got,
          "the same without the in-thread synchronize:", nosync)
    for name, bad in controls.items():
        assert all(b == 0 for row in bad for b in row), (name, bad)
    assert all(b == 0 for row in got for b in row), got
