"""Multi-process path on CPU (gloo, world_size 2): the sharding, the max-over-ranks
timing reduction and the SoA all-gather that bench.py and the IK callers use.
The per-shard compute here is the CPU oracle (test-only stand-in for the GPU
kernel, which needs a device); what is under test is the distribution logic."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ARM, ROOT, golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_per_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import kinhip
    from kinhip import dist as D
    try:
        ctx = D.init_from_env(backend="gloo")
        tree = O.parse_urdf_tree(golden("fetch.urdf"))
        ids = [tree.joint_id(n) for n in ARM]
        lo = [tree.joint_lower[i - 1] for i in ids]
        hi = [tree.joint_upper[i - 1] for i in ids]
        start, n = D.shard_range(n_per_rank, ctx.rank)
        Q = kinhip.uniform_configs(lo, hi, n, start=start, dtype=torch.float64)
        om = O.OracleMech(tree)
        gl = tree.link_id("gripper_link")
        pose, _ = om.fk_jac_batch(Q.numpy(), ids, gl, ids, n_threads=1)
        D.barrier(ctx)
        tmax = D.max_over_ranks(ctx, [float(ctx.rank + 1), -float(ctx.rank)])
        allp = D.all_gather_cols(ctx, torch.from_numpy(pose))
        allq = D.all_gather_cols(ctx, Q)
        s2, n2 = D.split_range(1001, ctx.rank, ctx.world)
        if ctx.rank == 0:
            q.put((tmax, allp.numpy(), allq.numpy(), (s2, n2)))
        else:
            q.put(("split", (s2, n2)))
        ctx.dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put(("error", repr(e)))
        raise


def test_two_rank_shards_match_single_process():
    import oracle as O
    import kinhip
    world, n = 2, 1536
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    errs = [r for r in res if r[0] == "error"]
    assert not errs, errs
    main = [r for r in res if r[0] != "split"][0]
    split = [r[1] for r in res if r[0] == "split"][0]
    tmax, allp, allq, split0 = main
    assert tmax == [2.0, 0.0]
    tree = O.parse_urdf_tree(golden("fetch.urdf"))
    ids = [tree.joint_id(n_) for n_ in ARM]
    lo = [tree.joint_lower[i - 1] for i in ids]
    hi = [tree.joint_upper[i - 1] for i in ids]
    Qfull = kinhip.uniform_configs(lo, hi, world * n, dtype=torch.float64).numpy()
    np.testing.assert_array_equal(allq, Qfull)
    ref, _ = O.OracleMech(tree).fk_jac_batch(Qfull, ids, tree.link_id("gripper_link"), ids)
    np.testing.assert_array_equal(allp, ref)
    assert split0 == (0, 501) and split == (501, 500)


def test_local_rank_beyond_the_gpus_is_refused(monkeypatch):
    """One process per GPU: LOCAL_RANK >= the visible GPU count raises instead of silently
    putting two ranks on one GPU; only the explicit gloo rehearsal may share a GPU."""
    import kinhip.dist as D
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.delenv("KINHIP_DIST_BACKEND", raising=False)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    with pytest.raises(RuntimeError, match="one process per GPU"):
        D.init_from_env()
    picked = []
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: picked.append(d))
    ctx = D.init_from_env(backend="gloo")  # rehearsal: ranks share GPU 0
    assert ctx.device == torch.device("cuda", 0) and picked == [torch.device("cuda", 0)]
