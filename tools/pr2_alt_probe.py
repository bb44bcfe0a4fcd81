"""Why does stage 2's restart attempt 1 from reset_manip_pose (kin_ik_coll_batch_alt) converge less often than
the same start as attempt 0?  bench.py _pr2_leg's batch (fp32): iteration histogram of stage 2 from the manip
pose alone, the step budget of one attempt, and the alt schedule at a few iteration budgets.
    python tools/pr2_alt_probe.py > gpurun_out/pr2_alt_probe.json"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

dev = torch.device("cuda", 0)
nt = 4096
dt = torch.float32
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "pr2_two_arms.urdf"), with_base=True)
joints = [m.find_joint(n) for n in kinhip.PR2_RARM_JOINTS + kinhip.PR2_LARM_JOINTS]
m.set_joint_angles([m.find_joint("torso_lift_joint")], [0.3, 0.0, 0.0, 0.0])
sscc = kinhip.SweptSphereCollisionChecker(m)
for name, c, r in kinhip.PR2_ARM_SPHERES:
    sscc.add_coll_sphere(m.find_link(name), c, r)
cplan = kinhip.CollisionIKPlan(sscc, m.find_link("l_gripper_tool_frame"), joints, dtype=dt).specialize()
rng = np.random.default_rng(29)
tg = np.zeros((12, nt))
for k in range(nt):
    yaw = rng.uniform(-0.2, 0.2)
    c, s_ = np.cos(yaw), np.sin(yaw)
    R = np.array([[c, -s_, 0.0], [s_, c, 0.0], [0.0, 0.0, 1.0]])
    tg[:, k] = np.concatenate([R.T.reshape(-1), [1.2 + rng.uniform(-0.06, 0.0), rng.uniform(-0.06, 0.06),
                                                 1.2 + rng.uniform(-0.05, 0.05)]])
doors = rng.uniform(1.6, 2.4, nt)
fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
asdf = kinhip.AttachedUnionSDF(fr, [fr.find_joint("door_joint")])
T = torch.tensor(tg, dtype=dt, device=dev).contiguous()
SQ = torch.zeros((4, nt), dtype=dt, device=dev)
SQ[0] = torch.tensor(doors, dtype=dt)
SQ[1] = 1.2
r, l, _ = kinhip.PR2_MANIP_POSE
q_manip = np.concatenate([np.deg2rad(np.array(r + l)), np.zeros(3)])
Q0 = torch.tensor(np.repeat(q_manip[:, None], nt, 1), dtype=dt, device=dev).contiguous()
out = {"targets": nt}
kw = dict(restarts=3, seed=1, with_rot=2)
Q1 = torch.empty_like(Q0)
cplan.ik_dls(T, Q1, Q0=Q0, max_iters=128, **kw)
# stage 2 from the manip pose alone, one long attempt: how many steps does it need?
_, it, _ = cplan.ik_coll(asdf, T, torch.empty_like(Q0), Q0=Q0, margin=0.02, scene_q=SQ, max_iters=256,
                         restarts=0, seed=1, with_rot=2)
it = it.cpu().numpy()
out["from_manip_one_attempt_256"] = {f"conv_within_{k}": float((it <= k).mean()) for k in (16, 24, 28, 30, 31, 32,
                                                                                           33, 40, 48, 64, 128, 256)}
# the schedules
for mi in (128, 132, 160, 192):
    for alt in (False, True):
        _, it2, _ = cplan.ik_coll(asdf, T, torch.empty_like(Q0), Q0=Q1, margin=0.02, scene_q=SQ, max_iters=mi,
                                  Q_alt=Q0 if alt else None, **kw)
        out[f"stage2_max_iters{mi}_{'alt' if alt else 'drawn'}"] = float((it2 <= mi).float().mean())
    _, it3, _ = cplan.ik_coll(asdf, T, torch.empty_like(Q0), Q0=Q0, margin=0.02, scene_q=SQ, max_iters=mi, **kw)
    out[f"stage2_from_manip_max_iters{mi}"] = float((it3 <= mi).float().mean())
print(json.dumps(out))
