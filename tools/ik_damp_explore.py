"""Config-4 IK on the oracle (CPU, fp64): success and iteration counts of the damped least squares with a
fixed lambda against the error-scaled damping lambda^2 + mu |e|^2 (Levenberg-Marquardt after Sugihara),
on config 4's targets (FK of seeded uniform configurations, q0 = 0), attempt 0 and the full schedule.
    python tools/ik_damp_explore.py [n] [with_rot]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
sys.path.insert(0, ROOT)
import kinhip  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
wr = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tree = O.parse_urdf_tree(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
mech = O.OracleMech(tree)
ids = [tree.joint_id(j) for j in kinhip.FETCH_ARM_JOINTS]
gl = tree.link_id("gripper_link")
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
arm = [m.find_joint(j) for j in kinhip.FETCH_ARM_JOINTS]
Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=4242,
                            dtype=__import__("torch").float64).numpy()
tgt = mech.fk_batch(Qt, ids, [gl])[0]
q0 = np.zeros((8, n))
grid = [(1e-2, 0.0, 0.5), (1e-2, 0.02, 0.5), (1e-2, 0.0, 1.0), (1e-2, 0.02, 1.0), (1e-2, 0.02, 0.75),
        (1e-2, 0.005, 0.5), (1e-2, 0.05, 0.5), (1e-2, 0.02, 0.35), (1e-2, 0.02, 1.5)]
if len(sys.argv) > 3:
    grid = [tuple(float(x) for x in g.split(",")) for g in sys.argv[3:]]
for lam, mu, ms in grid:
    _, it1, _ = mech.ik_dls_batch(q0, ids, gl, tgt, max_iters=16, lam=lam, with_rot=wr, damp_err=mu, max_step=ms)
    _, it4, _ = mech.ik_dls_batch(q0, ids, gl, tgt, max_iters=64, lam=lam, with_rot=wr, restarts=3, damp_err=mu,
                                  max_step=ms)
    c1 = it1 <= 16
    c10 = it1 <= 10
    c4 = it4 <= 64
    print(f"lam={lam:6.0e} mu={mu:5.3f} max_step={ms:4.2f}: attempt 0 solves {c1.mean():.4f} (by it 10: {c10.mean():.4f}), mean it "
          f"{it1[c1].mean():5.2f}; 64 it + 3 restarts: success {c4.mean():.4f}, mean it {it4[c4].mean():5.2f}",
          flush=True)
