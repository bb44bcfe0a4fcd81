"""Config-4 IK timing for one build / group setting (KINHIP_LIB, KINHIP_IK_GROUP select).
    python tools/ik_ab.py"""
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
out = []
for dt in ((torch.float32,) if os.environ.get("AB_F32") else (torch.float32, torch.float64)):
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt)
    if int(os.environ.get("AB_SPEC", "0")):
        plan.specialize()
    n = int(os.environ.get("IK_N", 65536))
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=4242,
                                dtype=dt, device=dev)
    tgt = plan.run(Qt)[0][0].contiguous()
    Q0 = torch.zeros((8, n), dtype=dt, device=dev)
    kw = dict(max_iters=64, restarts=3, seed=0, lam=1e-2, max_step=float(os.environ.get("IK_MAXSTEP", 0.5)),
              damp_err=float(os.environ.get("IK_DAMP", 0.0)), tol_pos=1e-3, tol_rot=1e-3)
    Qs = [Q0.clone() for _ in range(12)]
    plan.ik_dls(tgt, Qs[0], **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(1, 11):
        Q, it, err = plan.ik_dls(tgt, Qs[k], **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    out.append(f"{str(dt)[6:]}: {ms:.3f} ms/batch {n / ms * 1e3:.3e} solves/s succ {(it <= 64).float().mean():.4f} "
               f"mean_it {it.float().mean():.2f} qsum {float(Q.double().sum()):.6f}")
print(os.path.basename(os.environ.get("KINHIP_LIB", "default")), "G=" + os.environ.get("KINHIP_IK_GROUP", "auto"),
      "Q=" + os.environ.get("KINHIP_IK_QUEUE", "auto"), "spec=" + os.environ.get("AB_SPEC", "0"),
      f"max_step={kw['max_step']} damp_err={kw['damp_err']}",
      " | ".join(out), flush=True)
