"""Can two RCCL ranks share one GPU?  Spawns two ranks on cuda:0 with the "nccl" backend and runs one
all_gather_into_tensor; prints what RCCL says (the 1-GPU box cannot run a real multi-rank group).
usage: timeout -k 10 120 python tools/rccl_probe.py"""
import os
import socket

import torch
import torch.multiprocessing as mp


def _w(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        t = torch.full((4,), float(rank), device="cuda")
        out = torch.empty(8, device="cuda")
        dist.all_gather_into_tensor(out, t)
        torch.cuda.synchronize()
        q.put((rank, "ok", out.cpu().tolist()))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, "error", repr(e)[:400]))


if __name__ == "__main__":
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_w, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for _ in range(2):
        print(q.get(timeout=90), flush=True)
    for p in ps:
        p.join(timeout=30)
    print("exitcodes", [p.exitcode for p in ps])
