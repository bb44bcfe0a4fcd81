"""Row-padding probe: FK + J fp32 with the SoA rows (ldq / ldp / ldj) skewed off powers of two.
    python tools/ld_probe.py"""
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
plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32)
lo, hi = [j.lower_limit for j in arm], [j.upper_limit for j in arm]
for lg in (20, 22, 24):
    N = 1 << lg
    for pad in (0, 64, 96, 256, 1088, 4160):
        ld = N + pad
        Qb = torch.empty((8, ld), dtype=torch.float32, device=dev)
        Qb[:, :N] = kinhip.uniform_configs(lo, hi, N, dtype=torch.float32, device=dev)
        Q = Qb[:, :N]
        P = torch.empty((1, 12, ld), dtype=torch.float32, device=dev)[:, :, :N]
        J = torch.empty((8, 6, ld), dtype=torch.float32, device=dev)[:, :, :N]
        for _ in range(5):
            plan.run(Q, P, J)
        torch.cuda.synchronize()
        k = max(5, (1 << 26) // N)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(k):
            plan.run(Q, P, J)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / k * 1e3
        print(f"N=2^{lg} pad={pad:5d} floats: {us:8.2f} us  {272 * N / us / 1e3:7.1f} GB/s", flush=True)
        del Qb, P, J
