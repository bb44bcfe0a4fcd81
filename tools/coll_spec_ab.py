"""Config-5 k_coll timings on the specialised kernels (the bench's legs): min distance, distances +
gradients on plain SoA rows and on the tiled layout (tile 8192).  Knobs come from the environment
(KINHIP_COLL_PER_LANE, ...).   python tools/coll_spec_ab.py"""
import os
import sys
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
sdf = kinhip.fridge_sdf(fr)
sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
dt = torch.float32
cp = sscc.plan(arm, dtype=dt).specialize()
n = 1 << 20
Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=555, dtype=dt,
                           device=dev)
# the bench's f2 door sweep: boxes attached to the fridge, one door angle per sample
asdf = kinhip.AttachedUnionSDF(fr, [fr.find_joint("door_joint")])
g = torch.Generator().manual_seed(90)
SQ = torch.zeros((4, n), dtype=torch.float64)
SQ[0] = torch.rand(n, generator=g, dtype=torch.float64) * 2.4
SQ[1] = 1.2
SQ = SQ.to(dt).to(dev).contiguous()
res = []
for name, run in (("min", lambda: cp.run(sdf, Q, dists=False, min_dist=True)),
                  ("grad", lambda: cp.run(sdf, Q, dists=True, grads=True)),
                  ("scene", lambda: cp.run(asdf, Q, grads=True, min_dist=True, scene_q=SQ))):
    for _ in range(3):
        r = run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        r = run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    chk = float(r[2].double().sum()) if name == "min" else float(r[1].double().abs().sum())
    res.append(f"{name}: {us:6.1f}us chk {chk:.9e}")
print(" | ".join(res), flush=True)
