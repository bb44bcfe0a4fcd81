"""fp32 collision error vs the oracle on config 5's bench dataset (2^20 Fetch configurations, seed 555,
the fridge scene, 14 build-defined spheres): distances, min distance and 14x8 gradients of the
specialised kernel, plain and tiled, against the oracle at the fp32-rounded angles.  Prints the max
errors and, for the gradients, the error against the oracle's forward-difference gradient split by
the sphere centre's distance to the union (rho).  Run with KINHIP_LIB=.../libkinhip_ab.so and
KINHIP_COLL_FAST_TRIG=0|1 to compare hardware and exact trig.
    python tools/coll_fp32_err.py [log2 n]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("kinematics.jl_amd", "oracle", "tests", ""):
    sys.path.insert(0, os.path.join(ROOT, p))
import kinhip  # noqa: E402
import oracle as O  # noqa: E402
from bench import fridge_scene  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << lg
dev = torch.device("cuda", 0)
m, arm, sscc, sdf = fridge_scene()
Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, start=0, seed=555,
                           dtype=torch.float32, device=dev)
plan = sscc.plan(arm, dtype=torch.float32).specialize()
_, _, Mn = plan.run(sdf, Q, dists=False, min_dist=True)
D, G, Mn2 = plan.run(sdf, Q, grads=True, min_dist=True)
Dt, Gt, _ = plan.run_tiled(sdf, kinhip.tiled(Q, 8192), n, grads=True)
torch.cuda.synchronize()
tiled_equal = torch.equal(kinhip.untiled(Dt, n), D) and torch.equal(kinhip.untiled(Gt, n), G)

tree = O.parse_urdf_tree(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
om = O.OracleMech(tree)
sph, rad = [], []
for name, c, r in kinhip.FETCH_ARM_SPHERES:
    T = np.eye(4)
    T[:3, 3] = c
    sph.append(om.add_new_link(tree.link_id(name), T))
    rad.append(r)
fr = O.parse_urdf_tree(os.path.join(ROOT, "tests", "golden", "fridge.urdf"))
box = O.OracleUnionSDF(*O.fridge_boxes(fr))
ids = [tree.joint_id(x) for x in kinhip.FETCH_ARM_JOINTS]
t0 = time.time()
rd, rg = O.coll_batch(om, box, Q.double().cpu().numpy(), ids, sph, rad, n_threads=16)
t_or = time.time() - t0
d = D.double().cpu().numpy()
g = G.double().cpu().numpy()
ed = np.abs(d - rd)
em = np.abs(Mn.double().cpu().numpy() - rd.min(0))
em2 = np.abs(Mn2.double().cpu().numpy() - rd.min(0))
rho = np.abs(rd + np.asarray(rad)[:, None])  # |sdf(centre)|
eg = np.abs(g - rg)  # [sph, dof, n]
print(f"n={n} fast_trig={os.environ.get('KINHIP_COLL_FAST_TRIG', 'default')} lib={os.path.basename(kinhip.LIB_PATH)} "
      f"oracle {t_or:.1f}s tiled==plain {tiled_equal}")
print(f"dist max {ed.max():.3e} p99.99 {np.quantile(ed, 0.9999):.3e} p99 {np.quantile(ed, 0.99):.3e} | "
      f"min_dist (min-only kernel) max {em.max():.3e} | min_dist (grad kernel) max {em2.max():.3e}")
for lo_, hi_ in ((0, 1e-3), (1e-3, 1e-2), (1e-2, 0.05), (0.05, 0.2), (0.2, 10)):
    sel = (rho >= lo_) & (rho < hi_)
    if sel.any():
        e = eg.transpose(1, 0, 2)[:, sel]  # [dof, k]
        print(f"grad rho in [{lo_:g},{hi_:g}): {sel.sum()} sphere-samples, max {e.max():.3e}, "
              f"p99.99 {np.quantile(e, 0.9999):.3e}, frac>1e-5 {(e > 1e-5).mean():.2e}, frac>1e-4 {(e > 1e-4).mean():.2e}")
# the error scaled by the stated bound 5e-6 * (1 + 1 / rho)
bound = 5e-6 * (1.0 + 1.0 / np.maximum(rho, 1e-12))[:, None, :]
over = eg > bound
print(f"entries over 5e-6*(1+1/rho): {over.sum()} of {eg.size} ({over.mean():.2e})")
