"""Runs one engine workload K times for rocprofv3 (kernel trace / PMC passes).

    python tools/prof_kernel.py --what fkjac32 --steps 20
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

ap = argparse.ArgumentParser()
BASE = ["fkjac32", "fkjac32t", "fkjac64", "fkjac64t", "fk6_64", "fk6_64t", "ik32", "ik64", "coll32", "collg32", "collg32t",
        "coll64", "scene32", "cik32", "cikp32"]
ap.add_argument("--what", default="fkjac32", choices=BASE + [w + "s" for w in BASE],
                help="workload; a trailing 's' runs the plan-specialised kernels (kin_plan_specialize)")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--pad", type=int, default=256, help="row padding of the SoA buffers (as bench.py)")
ap.add_argument("--tile", type=int, default=8192, help="tile of the tiled-SoA workloads (*t, as bench.py)")
a = ap.parse_args()
SPEC = a.what.endswith("s")  # plan-specialised kernels (kin_plan_specialize)
if SPEC:
    a.what = a.what[:-1]
if a.what.endswith("64t") or a.what.endswith("64"):
    a.tile = a.tile // 2 if a.what.endswith("t") and a.tile == 8192 else a.tile  # fp64: same bytes per tile row
if a.what.startswith("ik") and a.n == 1 << 20:
    a.n = 65536  # config 4 size
dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
gl = m.find_link("gripper_link")
dt = torch.float64 if "64" in a.what else torch.float32
Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], a.n, dtype=dt, device=dev)
ld = a.n + a.pad
if a.what.startswith("fkjac") and a.what.endswith("t"):
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt)
    if SPEC:
        plan.specialize()
    Qt = kinhip.tiled(Q, a.tile)
    nt = Qt.shape[0]
    P = torch.empty((nt, 1, 12, a.tile), dtype=dt, device=dev)
    J = torch.empty((nt, 8, 6, a.tile), dtype=dt, device=dev)
    for _ in range(a.steps):
        plan.run_tiled(Qt, a.n, P, J)
elif a.what.startswith("fkjac"):
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt)
    if SPEC:
        plan.specialize()
    Qb = torch.empty((8, ld), dtype=dt, device=dev)
    Qb[:, :a.n] = Q
    Q = Qb[:, :a.n]
    P = torch.empty((1, 12, ld), dtype=dt, device=dev)[:, :, :a.n]
    J = torch.empty((8, 6, ld), dtype=dt, device=dev)[:, :, :a.n]
    for _ in range(a.steps):
        plan.run(Q, P, J)
elif a.what.startswith("fk6_64"):
    links = [m.find_link(n) for n in ["l_gripper_finger_link", "r_gripper_finger_link", "wrist_flex_link",
                                      "wrist_roll_link", "shoulder_lift_link", "upperarm_roll_link"]]
    plan = m.plan(arm, out_links=links, dtype=dt)
    if SPEC:
        plan.specialize()
    if a.what.endswith("t"):
        Qt = kinhip.tiled(Q, a.tile)
        P = torch.empty((Qt.shape[0], 6, 12, a.tile), dtype=dt, device=dev)
        for _ in range(a.steps):
            plan.run_tiled(Qt, a.n, P)
    else:
        P = torch.empty((6, 12, a.n), dtype=dt, device=dev)
        for _ in range(a.steps):
            plan.run(Q, P)
elif a.what == "scene32":  # bench f2_scene_door_sweep: boxes attached to the fridge, one door angle per sample
    fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
    asdf = kinhip.AttachedUnionSDF(fr, [fr.find_joint("door_joint")])
    sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
    cp = sscc.plan(arm, dtype=dt)
    if SPEC:
        cp.specialize()
        cp.specialize_scene(asdf)  # (as the bench's leg: the fridge's tables compiled in, kinhip_jit_collc_1)
    g = torch.Generator().manual_seed(90)
    SQ = torch.zeros((4, a.n), dtype=torch.float64)
    SQ[0] = torch.rand(a.n, generator=g, dtype=torch.float64) * 2.4
    SQ[1] = 1.2
    SQ = SQ.to(dt).to(dev).contiguous()
    for _ in range(a.steps):
        cp.run(asdf, Q, grads=True, min_dist=True, scene_q=SQ)
elif a.what == "cik32":  # bench f3_collision_ik: stage 2 (kin_ik_coll_batch) of 4,096 fridge targets
    import numpy as np
    fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
    sdf = kinhip.fridge_sdf(fr)
    sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
    nt = 4096
    rng = np.random.default_rng(17)
    tg = np.zeros((12, nt))
    for k in range(nt):
        x, y, z, yaw = rng.uniform(0.9, 1.05), rng.uniform(-0.12, 0.12), rng.uniform(1.15, 1.32), rng.uniform(-0.3, 0.3)
        c, s_ = np.cos(yaw), np.sin(yaw)
        tg[:, k] = np.concatenate([np.array([[c, -s_, 0.0], [s_, c, 0.0], [0.0, 0.0, 1.0]]).T.reshape(-1), [x, y, z]])
    tg = torch.tensor(tg, dtype=dt, device=dev).contiguous()
    cplan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=dt)
    if SPEC:
        cplan.specialize()
    Q0 = torch.zeros((8, nt), dtype=dt, device=dev)
    Q1 = torch.empty_like(Q0)
    kw = dict(max_iters=128, restarts=3, seed=1, with_rot=2)
    cplan.ik_dls(tg, Q1, Q0=Q0, **kw)
    for _ in range(a.steps):
        cplan.ik_coll(sdf, tg, torch.empty_like(Q1), Q0=Q1, margin=0.02, **kw)
elif a.what == "cikp32":  # bench f3_collision_ik_pillar_4096: stage 2 around a pillar on the elbow
    import numpy as np
    fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
    sdf0 = kinhip.fridge_sdf(fr)
    sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
    T0 = np.eye(4)
    T0[:3, 3] = (0.75, 0.15, 1.0)
    m.set_joint_angles(arm, np.zeros(8))
    kinhip.inverse_kinematics_(m, gl, arm, T0)
    P = np.eye(4)
    P[:3, 3] = kinhip.get_transform(m, m.find_link("elbow_flex_link"))[:3, 3]
    m.set_joint_angles(arm, np.zeros(8))
    sdf = kinhip.UnionSDF(sdf0.sdfs + [kinhip.BoxSDF(P, (0.08, 0.08, 0.08))])
    nt = 4096
    rng = np.random.default_rng(5)
    tg = np.zeros((12, nt))
    for k in range(nt):
        tg[:, k] = np.concatenate([np.eye(3).reshape(-1), T0[:3, 3] + rng.uniform(-0.005, 0.005, 3)])
    tg = torch.tensor(tg, dtype=dt, device=dev).contiguous()
    cplan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=dt)
    if SPEC:
        cplan.specialize()
    Q0 = torch.zeros((8, nt), dtype=dt, device=dev)
    Q1 = torch.empty_like(Q0)
    kw = dict(max_iters=128, restarts=3, seed=1, with_rot=2)
    cplan.ik_dls(tg, Q1, Q0=Q0, **kw)
    for _ in range(a.steps):
        cplan.ik_coll(sdf, tg, torch.empty_like(Q1), Q0=Q1, margin=0.02, **kw)
elif a.what.startswith("coll"):  # config 5: Fetch arm spheres vs the fridge scene
    fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
    sdf = kinhip.fridge_sdf(fr)
    sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
    cp = sscc.plan(arm, dtype=dt)
    if SPEC:
        cp.specialize()
    grads = a.what.startswith("collg")
    if grads:  # rows padded like the bench's plain leg (ld = n + pad)
        Qb = torch.empty((8, ld), dtype=dt, device=dev)
        Qb[:, :a.n] = Q
        Q = Qb[:, :a.n]
        D = torch.zeros((cp.n_sph, ld), dtype=dt, device=dev)[:, :a.n]
        G = torch.zeros((cp.n_sph, 8, ld), dtype=dt, device=dev)[:, :, :a.n]
        for _ in range(a.steps):
            cp.run(sdf, Q, dists=D, grads=G)
    else:
        for _ in range(a.steps):
            cp.run(sdf, Q, dists=False, min_dist=True)
else:
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt)
    if SPEC:
        plan.specialize()
    T, _ = plan.run(Q)
    tgt = T[0].contiguous()
    for _ in range(a.steps):
        Q0 = torch.zeros_like(Q)
        plan.ik_dls(tgt, Q0, max_iters=64, restarts=3, lam=1e-2, max_step=0.5)  # bench IK_KW
torch.cuda.synchronize()
print("done", a.what, a.steps)
