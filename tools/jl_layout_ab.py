"""FK + J fp32 (specialised) at 2^20 in the Julia shim's layout (plain SoA rows, ld = N) and padded
(ld = N + 256), warm: the A/B workload of tools/ab.py "jl" (KINHIP_FK_PER_LANE, KINHIP_JIT_DEFS, ...)."""
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
plan = m.plan(arm, out_links=[gl], jac_link=gl, jac_joints=arm, with_rot=True, dtype=torch.float32).specialize()
lo, hi = [j.lower_limit for j in arm], [j.upper_limit for j in arm]
N = 1 << 20
st = torch.cuda.Stream(dev)
out = []
for pad in (0, 256):
    Qb = torch.empty((8, N + pad), dtype=torch.float32, device=dev)
    Qb[:, :N] = kinhip.uniform_configs(lo, hi, N, dtype=torch.float32, device=dev)
    P = torch.zeros((1, 12, N + pad), dtype=torch.float32, device=dev)[:, :, :N]
    J = torch.zeros((8, 6, N + pad), dtype=torch.float32, device=dev)[:, :, :N]
    Q = Qb[:, :N]
    with torch.cuda.stream(st):
        for _ in range(10):
            plan.run(Q, P, J, stream=st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(50):
            plan.run(Q, P, J, stream=st)
        e1.record(st)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    out.append(f"ld=N+{pad}: {us:.2f} us ({272 * N / us / 1e3:.0f} GB/s) jsum {float(J.double().sum()):.6e}")
    del Qb, P, J
print(" | ".join(out), flush=True)
