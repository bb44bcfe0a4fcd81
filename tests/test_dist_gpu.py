"""Sharded path on the GPU: two ranks (gloo for the exchange, both on cuda:0, spawned as
fresh processes) run the real kinhip plans through bench.py's shard / gather helpers -- config 4's IK
targets and config 5's collision validity samples -- and the gathered results must be bit-identical to
one process solving the whole set.  (The RCCL backend is the same all_gather_into_tensor call; a
world-size-2 RCCL group needs two GPUs, which the 1-GPU test box does not have.)"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu

N_IK, N_COLL = 4096, 1 << 16  # per rank


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_results(ctx, bench):
    import kinhip
    m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
    arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
    gl = m.find_link("gripper_link")
    dt = torch.float32
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt, specialize=True)
    n_ik = N_IK * (2 if ctx.world == 1 else 1)  # the single process solves both shards
    tgt, kw = bench.ik_shard(m, arm, gl, ctx, n_ik, dt)
    Q, it, err = plan.ik_dls(tgt, torch.zeros((8, n_ik), dtype=dt, device=ctx.device), **kw)
    mf, armf, sscc, sdf = bench.fridge_scene()
    n_c = N_COLL * (2 if ctx.world == 1 else 1)
    Qc = bench.coll_shard(armf, ctx, n_c, dt)
    _, _, mn = sscc.plan(armf, dtype=dt, specialize=True).run(sdf, Qc, dists=False, min_dist=True)
    valid = (mn > 0).to(torch.uint8).reshape(1, -1)
    torch.cuda.synchronize()
    D = bench.D
    return (D.all_gather_cols(ctx, Q).cpu(), D.all_gather_cols(ctx, it.reshape(1, -1)).cpu(),
            D.all_gather_cols(ctx, err).cpu(), D.all_gather_cols(ctx, valid).cpu())


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import sys
    sys.path.insert(0, ROOT)
    try:
        import bench
        ctx = bench.D.init_from_env(backend="gloo")  # both ranks share GPU 0
        res = _shard_results(ctx, bench)
        if rank == 0:
            q.put(("ok", [r.numpy() for r in res]))
        bench.D.barrier(ctx)
        ctx.dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put(("error", repr(e)))
        raise


def test_two_ranks_on_gpu_match_one_process():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    world = 2
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    port = _free_port()
    procs = [mctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, payload = q.get(timeout=110)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", payload
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ctx1 = bench.D.init_from_env()  # world 1 (no torchrun variables in the test process)
    assert ctx1.world == 1
    ref = [r.numpy() for r in _shard_results(ctx1, bench)]
    for name, a, b in zip(("q", "iters", "err", "valid"), payload, ref):
        assert a.shape == b.shape, (name, a.shape, b.shape)
        np.testing.assert_array_equal(a, b, err_msg=name)
    assert (ref[1] <= 64).mean() > 0.99  # the IK set solves (kinhip.h: iters > max_iters = failure)


def _rccl_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import sys
    sys.path.insert(0, ROOT)
    try:
        import bench
        ctx = bench.D.init_from_env(backend="nccl", always_group=True)  # RCCL on ROCm
        assert ctx.dist.get_backend() == "nccl", ctx.dist.get_backend()
        res = _shard_results(ctx, bench)  # all_gather_into_tensor on device memory
        mx = bench.D.max_over_ranks(ctx, [1.5, -2.0])  # all_reduce(MAX) of a device fp64 tensor
        bench.D.barrier(ctx)
        q.put(("ok", [r.numpy() for r in res], mx))
        ctx.dist.destroy_process_group()
    except Exception as e:
        q.put(("error", repr(e), None))
        raise


def test_rccl_collectives_of_the_sharded_path():
    """The RCCL ("nccl") backend itself: a one-rank group runs the bench's device-memory all-gathers,
    the max-over-ranks all-reduce and the barrier; the gathered IK / collision results equal the
    group-free run bit for bit.  (World size 1: the test box has one GPU.)"""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    p = mctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    status, payload, mx = q.get(timeout=110)
    p.join(timeout=60)
    assert status == "ok", payload
    assert p.exitcode == 0, p.exitcode
    assert mx == [1.5, -2.0]
    ref = [r.numpy() for r in _shard_results(bench.D.init_from_env(), bench)]
    for name, a, b in zip(("q", "iters", "err", "valid"), payload, ref):
        np.testing.assert_array_equal(a, b, err_msg=name)
