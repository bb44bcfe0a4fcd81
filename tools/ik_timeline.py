"""Where config 4's time goes between launches: per-lane entry / write times (s_memrealtime, 100 MHz;
diagnostic A/B build, KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=9) of the two-phase solve, specialised fp32.
    KINHIP_LIB=.../libkinhip_ab.so KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=9 python tools/ik_timeline.py"""
import os
import sys
import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
gl = m.find_link("gripper_link")
plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32).specialize()
n = 65536
Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=4242,
                            dtype=torch.float32, device=dev)
tgt = plan.run(Qt)[0][0].contiguous()
Q0 = torch.zeros((8, n), dtype=torch.float32, device=dev)
kw = dict(max_iters=64, restarts=3, seed=0, lam=1e-2, max_step=float(os.environ.get("IK_MAXSTEP", 0.5)),
          damp_err=float(os.environ.get("IK_DAMP", 0.0)), tol_pos=1e-3, tol_rot=1e-3)
print(f"max_step {kw['max_step']} damp_err {kw['damp_err']}")
Q = Q0.clone()
for _ in range(5):
    _, it, err = plan.ik_dls(tgt, Q, Q0=Q0, **kw)
torch.cuda.synchronize()
ent = err[0].view(torch.int32).cpu().numpy().astype(np.int64) & 0xffffffff
ext = err[1].view(torch.int32).cpu().numpy().astype(np.int64) & 0xffffffff
it = it.cpu().numpy()
t0 = ent.min()
ent = (ent - t0) * 10.0 / 1000  # us
ext = (ext - t0) * 10.0 / 1000
p1 = it <= 10
for name, sel in (("phase 1 (written by phase 1)", p1), ("phase 2 (handed over)", ~p1)):
    e, x = ent[sel], ext[sel]
    print(f"{name}: {sel.sum()} targets; entry {e.min():.1f}..{e.max():.1f} us (p50 {np.median(e):.1f}); "
          f"write {x.min():.1f}..{x.max():.1f} us (p50 {np.median(x):.1f}); lane span p50 {np.median(x - e):.1f} "
          f"max {np.max(x - e):.1f} us")
print("iters histogram:", np.bincount(np.minimum(it, 65))[:20].tolist())
for k in range(3, 65):
    sel = it == k
    if sel.sum() >= 20:
        print(f"  iters {k:2d}: {sel.sum():6d} targets, write p50 {np.median(ext[sel]):6.1f} us, p90 {np.percentile(ext[sel], 90):6.1f}")
