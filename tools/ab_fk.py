"""One k_fk build variant's timings (KINHIP_LIB selects the build): FK + 6x8 J of Fetch gripper_link,
2^20 configurations, fp32 and fp64, plain SoA rows padded by 256 and tiled SoA (tile 4096).
usage: KINHIP_LIB=... python tools/ab_fk.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
gl = m.find_link("gripper_link")
lo, hi = [j.lower_limit for j in arm], [j.upper_limit for j in arm]
N = 1 << 20
res = []


def timed(fn, k=100):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k * 1e3


import time
SPEC = int(os.environ.get("AB_SPEC", "0"))
for dt, esz in ((torch.float32, 4), (torch.float64, 8)):
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt)
    if SPEC:
        t0 = time.perf_counter()
        plan.specialize()
        res.append(f"spec {time.perf_counter() - t0:.2f}s")
    Q = kinhip.uniform_configs(lo, hi, N, dtype=dt, device=dev)
    ld = N + 256
    Qb = torch.empty((8, ld), dtype=dt, device=dev)
    Qb[:, :N] = Q
    P = torch.empty((1, 12, ld), dtype=dt, device=dev)[:, :, :N]
    J = torch.empty((8, 6, ld), dtype=dt, device=dev)[:, :, :N]
    us = timed(lambda: plan.run(Qb[:, :N], P, J))
    res.append(f"{esz * 8}b soa+256 {us:6.2f}us")
    del Qb, P, J
    Qt = kinhip.tiled(Q, 4096)
    Pt = torch.empty((N // 4096, 1, 12, 4096), dtype=dt, device=dev)
    Jt = torch.empty((N // 4096, 8, 6, 4096), dtype=dt, device=dev)
    us = timed(lambda: plan.run_tiled(Qt, N, Pt, Jt))
    res.append(f"tile4096 {us:6.2f}us {68 * esz * N / us / 1e3:5.0f}GB/s")
    del Qt, Pt, Jt
print((os.path.basename(os.environ.get("KINHIP_LIB", "default")) + (" spec" if SPEC else "")).ljust(20), " | ".join(res), flush=True)
