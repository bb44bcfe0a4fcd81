"""Config-4 parameter exploration on the GPU: success rate and solves/s of the batched DLS IK
for Fetch gripper_link, 65,536 reachable targets (FK of seeded random q), q0 = 0."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
gl = m.find_link("gripper_link")
N = 65536
for dt in (torch.float32, torch.float64):
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt)
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, seed=4242, dtype=dt,
                                device=dev)
    tgt = plan.run(Qt)[0][0].contiguous()
    for iters, restarts, lam, step in [(64, 0, 1e-2, 0.5), (64, 1, 1e-2, 0.5), (64, 3, 1e-2, 0.5),
                                        (64, 1, 5e-2, 0.5), (64, 1, 1e-2, 0.3), (128, 3, 1e-2, 0.5),
                                        (256, 7, 1e-2, 0.5)]:
        Q = torch.zeros((8, N), dtype=dt, device=dev)
        plan.ik_dls(tgt, Q.clone(), max_iters=iters, restarts=restarts, lam=lam, max_step=step)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        K = 5
        for _ in range(K):
            Q2 = Q.clone()
            Q2, it, err = plan.ik_dls(tgt, Q2, max_iters=iters, restarts=restarts, lam=lam, max_step=step)
        torch.cuda.synchronize()
        dt_s = (time.perf_counter() - t0) / K
        conv = (it < iters).float().mean().item()
        print(json.dumps({"dtype": str(dt), "iters": iters, "restarts": restarts, "lam": lam, "max_step": step,
                          "success": round(conv, 4), "ms": round(dt_s * 1e3, 3), "solves_per_s": N / dt_s,
                          "mean_iters": it.float().mean().item()}))
