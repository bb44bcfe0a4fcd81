"""The bench's f3 leg (bistage collision-aware IK, 4,096 fridge targets, fp32, specialised) split by
stage: HIP-event time of stage 1 (kin_ik_dls_batch_from) and stage 2 (kin_ik_coll_batch), and the
iteration histograms of both.   python tools/cik_bench.py [N]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import kinhip  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dev = torch.device("cuda", 0)
dt = torch.float32
m, arm, sscc, sdf = bench.fridge_scene()
gl = m.find_link("gripper_link")
rng = np.random.default_rng(17)
tg = np.zeros((12, N))
for k in range(N):
    x, y, z, yaw = rng.uniform(0.9, 1.05), rng.uniform(-0.12, 0.12), rng.uniform(1.15, 1.32), rng.uniform(-0.3, 0.3)
    c, s = np.cos(yaw), np.sin(yaw)
    tg[:, k] = np.concatenate([np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]]).T.reshape(-1), [x, y, z]])
tg = torch.tensor(tg, dtype=dt, device=dev).contiguous()
plan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=dt).specialize()
Q0 = torch.zeros((8, N), dtype=dt, device=dev)
kw = dict(max_iters=128, restarts=3, seed=1, with_rot=2)
for rep in range(3):
    for lanes in (1, 0):  # stage 2: attempts in sequence on one lane / side by side (auto: 4 lanes)
        Q1 = torch.empty_like(Q0)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        _, it1, _ = plan.ik_dls(tg, Q1, Q0=Q0, **kw)
        e[1].record()
        Q2, it2, err = plan.ik_coll(sdf, tg, Q1, margin=0.02, lanes=lanes, **kw)
        e[2].record()
        torch.cuda.synchronize()
        print(f"N={N} stage1 {e[0].elapsed_time(e[1]) * 1e3:.1f} us  stage2 (lanes={lanes}) "
              f"{e[1].elapsed_time(e[2]) * 1e3:.1f} us", flush=True)
for name, it in (("stage1", it1), ("stage2", it2)):
    h = np.bincount(np.minimum(it.cpu().numpy(), 129), minlength=130)
    nz = {i: int(v) for i, v in enumerate(h) if v}
    print(name, "iterations histogram", nz)
print("stage2 converged", float((it2 <= 128).float().mean()), "min dist", float(err[2][it2 <= 128].min()))
