"""FK legs for A/B of compile-time variants (KINHIP_JIT_DEFS): the headline FK + 6x8 J fp32 (tile 8192)
and config 2 (FK of 6 links, fp64, tile 4096), 2^20 configurations, specialised kernels.
    python tools/fk_legs_ab.py"""
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
six = [m.find_link(n) for n in ["l_gripper_finger_link", "r_gripper_finger_link", "wrist_flex_link", "wrist_roll_link",
                                "shoulder_lift_link", "upperarm_roll_link"]]
n = 1 << 20
res = []
legs = [("fkjac32", torch.float32, [gl], True, 8192, n), ("fk6_64", torch.float64, six, False, 4096, n)]
if os.environ.get("FK_BIG"):  # 4x and 16x the Infinity Cache
    legs += [("fkjac32_2^22", torch.float32, [gl], True, 8192, 1 << 22), ("fkjac32_2^24", torch.float32, [gl], True, 8192, 1 << 24)]
for name, dt, links, jac, tile, n in legs:
    plan = m.plan(arm, out_links=links, jac_link=gl if jac else None, dtype=dt).specialize(kinhip.KIN_SPEC_FK)
    Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, dtype=dt, device=dev)
    Qt = kinhip.tiled(Q, tile)
    P = torch.zeros((Qt.shape[0], len(links), 12, tile), dtype=dt, device=dev)
    J = torch.zeros((Qt.shape[0], 8, 6, tile), dtype=dt, device=dev) if jac else None
    for _ in range(3):
        plan.run_tiled(Qt, n, P, J)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    reps = 30 if n <= 1 << 20 else 10
    for _ in range(reps):
        plan.run_tiled(Qt, n, P, J)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    res.append(f"{name}: {us:6.1f}us chk {float(P.double().sum()):.9e}")
    del Q, Qt, P, J
print("defs", os.environ.get("KINHIP_JIT_DEFS", "-"), "lds", os.environ.get("KINHIP_FK_LDS", "-"), " | ".join(res),
      flush=True)
