"""FK + 6x8 J fp32 (the headline workload, specialised kernel, tile 8192): warm back-to-back launches
at 2^20 and 2^24, and cold launches at 2^20 (each after a 1 GiB read).  KINHIP_FK_PER_LANE selects
the grid-strided variant; FK_AB_F64=1 runs the fp64 plan (tile 4096).   python tools/fk_stride_ab.py"""
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
DT = torch.float64 if os.environ.get("FK_AB_F64") else torch.float32
TILE = 4096 if DT == torch.float64 else 8192
plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=DT).specialize(kinhip.KIN_SPEC_FK)
res = []
scrub = torch.ones(1 << 28, dtype=torch.float32, device=dev)
ref = None
for lg in (20, 22, 24, 26):
    n = 1 << lg
    Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, dtype=DT,
                               device=dev)
    Qt = kinhip.tiled(Q, TILE)
    P = torch.zeros((Qt.shape[0], 1, 12, TILE), dtype=DT, device=dev)
    J = torch.zeros((Qt.shape[0], 8, 6, TILE), dtype=DT, device=dev)
    steps = 50 if lg == 20 else 10
    for _ in range(3):
        plan.run_tiled(Qt, n, P, J)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        plan.run_tiled(Qt, n, P, J)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / steps * 1e3
    res.append(f"2^{lg}: {us:7.1f}us {(272 if DT == torch.float32 else 544) * n / us / 1e3:6.0f}GB/s")
    if lg == 20:
        ref = (P.clone(), J.clone())
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            scrub.sum()
            a.record()
            plan.run_tiled(Qt, n, P, J)
            b.record()
        torch.cuda.synchronize()
        cu = sum(a.elapsed_time(b) for a, b in ev) / 10 * 1e3
        res.append(f"2^20 cold: {cu:6.1f}us")
        res.append(f"chk {float(P.double().sum()):.9e} {float(J.double().abs().sum()):.9e}")
    del Q, Qt, P, J
print("fk per_lane", os.environ.get("KINHIP_FK_PER_LANE", "1"), " | ".join(res), flush=True)
