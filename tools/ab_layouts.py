"""Layout scan for one FK workload on the plan-specialised kernel: plain SoA (ld = N + pad) vs
tiled SoA (tile T).  usage: python tools/ab_layouts.py [fk6_64|fkjac64|fkjac32]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "fk6_64"
dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
gl = m.find_link("gripper_link")
dt = torch.float64 if "64" in what else torch.float32
esz = 8 if dt == torch.float64 else 4
if what.startswith("fk6"):
    links = [m.find_link(n) for n in ["l_gripper_finger_link", "r_gripper_finger_link", "wrist_flex_link",
                                      "wrist_roll_link", "shoulder_lift_link", "upperarm_roll_link"]]
    plan = m.plan(arm, out_links=links, dtype=dt).specialize()
    rows_out, jac = 72, False
else:
    links = [gl]
    plan = m.plan(arm, out_links=links, jac_link=gl, dtype=dt).specialize()
    rows_out, jac = 60, True
N = 1 << 20
Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, dtype=dt, device=dev)


def timed(fn, k=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k * 1e3


res = []
nb = (8 + rows_out) * esz * N
for pad in (0, 256, 1024):
    ld = N + pad
    Qb = torch.empty((8, ld), dtype=dt, device=dev)
    Qb[:, :N] = Q
    P = torch.empty((len(links), 12, ld), dtype=dt, device=dev)[:, :, :N]
    J = torch.empty((8, 6, ld), dtype=dt, device=dev)[:, :, :N] if jac else None
    us = timed(lambda: plan.run(Qb[:, :N], P, J))
    res.append(f"soa+{pad} {us:6.1f}us {nb / us / 1e3:5.0f}")
    del Qb, P, J
for tile in (1024, 2048, 4096, 8192, 16384):
    Qt = kinhip.tiled(Q, tile)
    nt = Qt.shape[0]
    P = torch.empty((nt, len(links), 12, tile), dtype=dt, device=dev)
    J = torch.empty((nt, 8, 6, tile), dtype=dt, device=dev) if jac else None
    us = timed(lambda: plan.run_tiled(Qt, N, P, J))
    res.append(f"t{tile} {us:6.1f}us {nb / us / 1e3:5.0f}")
    del Qt, P, J
print(what, " | ".join(res), flush=True)
