"""Config-5 k_coll timings for one build (KINHIP_LIB selects it): min distance and distances + gradients."""
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
res = []
for dt in (torch.float32, torch.float64):
    cp = sscc.plan(arm, dtype=dt)
    n = 1 << 20
    Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=555, dtype=dt,
                               device=dev)
    pad = int(os.environ.get("COLL_PAD", "0"))
    Db = torch.empty((cp.n_sph, n + pad), dtype=dt, device=dev)[:, :n]
    Gb = torch.empty((cp.n_sph, cp.n_dof, n + pad), dtype=dt, device=dev)[:, :, :n]
    for name, kw in (("min", dict(dists=False, min_dist=True)), ("grad", dict(dists=Db, grads=Gb))):
        for _ in range(3):
            r = cp.run(sdf, Q, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            r = cp.run(sdf, Q, **kw)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        chk = float(r[2].double().sum()) if name == "min" else float(r[1].double().abs().sum())
        res.append(f"{str(dt)[6:]}-{name}: {us:7.1f}us chk {chk:.6e}")
print(os.path.basename(os.environ.get("KINHIP_LIB", "default")).ljust(20), "pad", os.environ.get("COLL_PAD", "0"),
      " | ".join(res), flush=True)
