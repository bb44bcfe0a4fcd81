"""One process per GPU.

Configurations are independent, so the batch path shards with no data-path
collective: rank r evaluates its own slice of one global counter-hashed
dataset (weak scaling: a fixed slice per GPU).  The only exchange is for
callers that need every result on one rank (IK solutions + status, collision
flags): an all-gather of the small per-configuration results over RCCL
(torch.distributed "nccl" on ROCm, point-to-point xGMI), never of the
272-byte-per-configuration FK+J output.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch


@dataclass
class Ctx:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    dist: Optional[object]  # torch.distributed when world > 1
    backend: str = "none"


def init_from_env(backend: Optional[str] = None, always_group: bool = False) -> Ctx:
    """torchrun / torch.distributed.run environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*).
    `always_group`: create the process group even at world size 1 (the single-GPU test box runs the
    RCCL collectives of the sharded path this way; a multi-rank RCCL group needs one GPU per rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = backend or os.environ.get("KINHIP_DIST_BACKEND")  # "gloo": rehearse ranks sharing one GPU
    use_cuda = torch.cuda.is_available()
    dev = torch.device("cpu")
    if use_cuda:
        ndev = torch.cuda.device_count()
        if local >= ndev:
            # one process per GPU: more local ranks than GPUs would silently double up GPUs.  Only the
            # explicit gloo rehearsal (KINHIP_DIST_BACKEND=gloo: ranks sharing one GPU) may do that.
            if backend != "gloo":
                raise RuntimeError(f"LOCAL_RANK {local} >= {ndev} visible GPUs: launch one process per GPU "
                                   f"(or set KINHIP_DIST_BACKEND=gloo to rehearse ranks sharing a GPU)")
            local_dev = local % max(1, ndev)
        else:
            local_dev = local
        dev = torch.device("cuda", local_dev)
        torch.cuda.set_device(dev)
    d, be = None, "none"
    if world > 1 or always_group:
        import torch.distributed as dist
        be = backend or ("nccl" if use_cuda else "gloo")
        if not dist.is_initialized():
            if be == "nccl":
                dist.init_process_group(be, device_id=dev)
            else:
                dist.init_process_group(be)
        d = dist
    return Ctx(rank, world, local, dev, d, be)


def _coll(ctx: Ctx, t: torch.Tensor) -> torch.Tensor:
    """Tensor placement for a collective: RCCL works on device memory, gloo on host memory."""
    return t.cpu() if ctx.backend == "gloo" else t


def shard_range(n_per_rank: int, rank: int) -> tuple[int, int]:
    """Weak scaling: rank r owns global configurations [r*n, (r+1)*n)."""
    return rank * n_per_rank, n_per_rank


def split_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Strong scaling: contiguous near-equal split of n_total configurations."""
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def barrier(ctx: Ctx):
    if ctx.dist is not None:
        ctx.dist.barrier()


def max_over_ranks(ctx: Ctx, values) -> list:
    """Element-wise max of a list of floats over ranks (timing: the slowest rank defines the job time)."""
    t = _coll(ctx, torch.tensor(list(values), dtype=torch.float64, device=ctx.device))
    if ctx.dist is not None:
        ctx.dist.all_reduce(t, op=ctx.dist.ReduceOp.MAX)
    return t.tolist()


def all_gather_cols(ctx: Ctx, local: torch.Tensor) -> torch.Tensor:
    """Gather SoA results sharded along the configuration axis: (k, n) on every rank ->
    (k, world*n) in rank order (equal shard sizes).  One RCCL all-gather."""
    if ctx.dist is None:
        return local
    k = local.shape[0]
    flat = _coll(ctx, local.contiguous().reshape(-1))
    out = torch.empty(ctx.world * flat.numel(), dtype=local.dtype, device=flat.device)
    ctx.dist.all_gather_into_tensor(out, flat)
    return out.reshape(ctx.world, k, -1).permute(1, 0, 2).reshape(k, -1).to(local.device)
