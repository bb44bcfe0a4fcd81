"""Probe for tests/test_gpu_collision_ik.py: a pillar placed on the elbow of the collision-free IK
solution, then the bistage solve must keep the pose and move the arm off the pillar."""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np, torch, kinhip
from conftest import ARM, golden
m = kinhip.parse_urdf(golden("fetch.urdf"))
fr = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
sdf0 = kinhip.fridge_sdf(fr)
sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
arm = [m.find_joint(n) for n in ARM]
gl = m.find_link("gripper_link")
for tgt in [(0.75, 0.15, 1.0), (0.7, -0.2, 1.1), (0.8, 0.0, 1.2), (0.6, 0.3, 0.9), (1.0, 0.0, 1.25)]:
    for link, size in [("elbow_flex_link", 0.08), ("upperarm_roll_link", 0.08), ("forearm_roll_link", 0.06)]:
        T = np.eye(4); T[:3, 3] = tgt
        m.set_joint_angles(arm, np.zeros(8))
        q1, st1 = kinhip.inverse_kinematics_(m, gl, arm, T)
        pe = kinhip.get_transform(m, m.find_link(link))[:3, 3]
        P = np.eye(4); P[:3, 3] = pe
        sdf = kinhip.UnionSDF(sdf0.sdfs + [kinhip.BoxSDF(P, (size, size, size))])
        d1 = kinhip.compute_coll_dists(sscc, arm, sdf)
        m.set_joint_angles(arm, np.zeros(8))
        t0 = time.time()
        q, st = kinhip.inverse_kinematics_(m, gl, arm, T, sscc, sdf, use_bistage=True)
        d = kinhip.compute_coll_dists(sscc, arm, sdf)
        Tn = kinhip.get_transform(m, gl)
        r = kinhip.rpy(Tn) - kinhip.rpy(T)
        good = st == ":FTOL_REACHED" and np.linalg.norm(Tn[:3, 3] - T[:3, 3]) < 1e-3 and np.linalg.norm(r) < 1e-3 and d.min() >= 0.02 - 1e-6
        print(tgt, link, st1, f"stage1 min {d1.min():.4f} ->", st, f"min {d.min():.4f} dp {np.linalg.norm(Tn[:3,3]-T[:3,3]):.1e} drpy {np.linalg.norm(r):.1e} {time.time()-t0:.2f}s", good, flush=True)
