"""How far the fp32 specialised IK (config-4 settings) sits from the fp64 oracle restatement:
iterates after k iterations (tol 0, no restarts) and final answers of targets both solve with equal
iteration counts.  python tools/ik_fp32_vs_fp64.py"""
import os
import sys
import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import kinhip  # noqa: E402
import oracle as O  # noqa: E402

dev = torch.device("cuda", 0)
urdf = os.path.join(ROOT, "tests", "golden", "fetch.urdf")
m = kinhip.parse_urdf(urdf)
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
gl = m.find_link("gripper_link")
tree = O.parse_urdf_tree(urdf)
om = O.OracleMech(tree)
ids = [j.id for j in arm]
N = 4096
lo = np.nan_to_num(np.array([j.lower_limit for j in arm]), neginf=-np.pi)
hi = np.nan_to_num(np.array([j.upper_limit for j in arm]), posinf=np.pi)
rng = np.random.default_rng(11)
qt = lo[:, None] + (hi - lo)[:, None] * rng.random((8, N))
tgt = om.fk_batch(qt, ids, [gl.id])[0]
t32 = torch.tensor(tgt, dtype=torch.float32, device=dev).contiguous()
plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32).specialize()
tgt32 = t32.double().cpu().numpy()  # the oracle sees the fp32-rounded targets
for k in (1, 2, 3, 5, 8):
    kw = dict(max_iters=k, restarts=0, seed=0, lam=1e-2, max_step=0.5, tol_pos=0.0, tol_rot=0.0)
    Q, _, _ = plan.ik_dls(t32, torch.zeros((8, N), dtype=torch.float32, device=dev), **kw)
    rq, _, _ = om.ik_dls_batch(np.zeros((8, N)), ids, gl.id, tgt32, n_threads=8, **kw)
    d = np.abs(Q.double().cpu().numpy() - rq).max(0)
    print(f"after {k} iterations: |q32 - q64| max {d.max():.2e} p99 {np.percentile(d, 99):.2e} p50 {np.median(d):.2e}")
kw = dict(max_iters=64, restarts=3, seed=0, lam=1e-2, max_step=0.5, tol_pos=1e-3, tol_rot=1e-3)
Q, it, _ = plan.ik_dls(t32, torch.zeros((8, N), dtype=torch.float32, device=dev), **kw)
rq, rit, _ = om.ik_dls_batch(np.zeros((8, N)), ids, gl.id, tgt32, n_threads=8, **kw)
it = it.cpu().numpy()
same = (it == rit) & (it <= 64)
d = np.abs(Q.double().cpu().numpy() - rq).max(0)
print(f"config-4 settings: converged fp32 {np.mean(it <= 64):.4f} fp64 {np.mean(rit <= 64):.4f}; equal iteration counts "
      f"{same.mean():.4f}; on those |q32 - q64| max {d[same].max():.2e} p99 {np.percentile(d[same], 99):.2e} "
      f"p50 {np.median(d[same]):.2e}; other targets {np.sum(~same)}")
