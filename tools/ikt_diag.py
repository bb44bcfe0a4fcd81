"""Where k_ik_tree (fp64, generic) and the oracle restatement part: the scenes of
tests/test_gpu_collision_ik{,_tree}.py run for k = 0, 1, 2, 4, 8 iterations without restarts (the first
iteration that differs), then with the tests' settings (the targets whose iteration counts differ).
    python tools/ikt_diag.py [scene ...]   scenes: fridge head twoarm twoarm_base"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
sys.path.insert(0, ROOT)
import kinhip  # noqa: E402
import oracle as O  # noqa: E402
import test_gpu_collision_ik_tree as T  # noqa: E402
from conftest import ARM, golden  # noqa: E402

dev = torch.device("cuda", 0)
np.set_printoptions(precision=6, linewidth=180, suppress=True)


def scene(name):
    if name in ("fridge", "head"):
        names = ARM + (["head_pan_joint", "head_tilt_joint"] if name == "head" else [])
        spheres = kinhip.FETCH_ARM_SPHERES + ([("head_pan_link", (0.1, 0.0, 0.1), 0.1),
                                               ("head_tilt_link", (0.05, 0.0, 0.0), 0.09),
                                               ("head_tilt_link", (0.15, 0.0, 0.0), 0.06)] if name == "head" else [])
        sc = T.Scene(golden("fetch.urdf"), names, spheres)
        rng = np.random.default_rng(41 if name == "head" else 23)
        N = 256 if name == "head" else 512
        tg = T._fridge_targets(rng, N)
        Q1 = T._stage1(sc, "gripper_link", tg, dev)
        sdf0, _ = T._fridge_box()
        if name == "head":
            c = sc.sphere_centres(Q1[:, 0].cpu().numpy(), None)[-2]
            sdf = kinhip.UnionSDF(sdf0.sdfs + [kinhip.BoxSDF(T._pose(c + [0.0, 0.0, 0.05]), (0.12, 0.3, 0.12))])
        else:
            sdf = sdf0
        return sc, "gripper_link", tg, Q1, sdf
    base = name == "twoarm_base"
    path = "/tmp/twoarm.urdf"
    with open(path, "w") as f:
        f.write(T.TWO_ARM)
    sc = T.Scene(path, T.TWO_ARM_Q, T.TWO_ARM_SPHERES, with_base=base)
    rng = np.random.default_rng(43)
    N = 300
    tg = np.zeros((12, N))
    for k in range(N):
        tg[:, k] = T._col(T._pose((rng.uniform(0.35, 0.55), rng.uniform(0.15, 0.35), rng.uniform(0.95, 1.2)),
                                  rng.uniform(-0.4, 0.4)))
    Q1 = T._stage1(sc, "l_grip", tg, dev)
    Q1[:4] = torch.tensor([0.3, 0.4, 0.0, 0.6], dtype=torch.float64, device=dev)[:, None]
    c = sc.sphere_centres(Q1[:, 0].cpu().numpy(), None)[6]
    sdf = kinhip.UnionSDF([kinhip.BoxSDF(T._pose(c), (0.1, 0.1, 0.1)),
                           kinhip.BoxSDF(T._pose((0.6, 0.0, 0.4)), (0.8, 1.2, 0.05))])
    return sc, "l_grip", tg, Q1, sdf


def run(sc, link, tg, Q1, sdf, kw):
    plan = kinhip.CollisionIKPlan(sc.sscc, sc.m.find_link(link), sc.q, dtype=torch.float64)
    tgt = torch.tensor(tg, dtype=torch.float64, device=dev).contiguous()
    Q, it, err = plan.ik_coll(sdf, tgt, torch.empty_like(Q1), Q0=Q1, lanes=1, **kw)
    box = O.OracleUnionSDF([b.pose for b in sdf.sdfs], [b.width for b in sdf.sdfs])
    rq, rit, rerr = O.ik_coll_batch(sc.om, box, Q1.cpu().numpy(), sc.ids, sc.tree.link_id(link), tg, sc.sph, sc.rad,
                                    sphere_parents=sc.par, **kw)
    return Q.cpu().numpy(), it.cpu().numpy(), err.cpu().numpy(), rq, rit, rerr


for name in (sys.argv[1:] or ["twoarm", "twoarm_base", "head", "fridge"]):
    sc, link, tg, Q1, sdf = scene(name)
    print(f"== {name}: q {len(sc.q)} cols, nd {sc.nd}, spheres {len(sc.sph)}", flush=True)
    for k in (0, 1, 2, 4, 8):
        kw = dict(T.KW, max_iters=k, restarts=0, tol_pos=0.0, tol_rot=0.0)
        q, it, e, rq, rit, re = run(sc, link, tg, Q1, sdf, kw)
        dq = np.abs(q - rq).max(0)
        de = np.abs(e - re).max(0)
        bad = np.where((dq > 1e-9) | (de > 1e-9))[0]
        print(f" k={k}: max |dq| {dq.max():.3e}, max |derr| {de.max():.3e}, targets off {bad.size}", flush=True)
        if bad.size and k <= 1:
            j = bad[0]
            print(f"   target {j}: q1 {Q1[:, j].cpu().numpy()}\n   gpu q {q[:, j]}\n   orc q {rq[:, j]}\n"
                  f"   gpu err {e[:, j]}\n   orc err {re[:, j]}", flush=True)
    q, it, e, rq, rit, re = run(sc, link, tg, Q1, sdf, T.KW)
    bad = np.where(it != rit)[0]
    print(f" test settings: converged gpu {np.mean(it <= T.KW['max_iters']):.3f} oracle "
          f"{np.mean(rit <= T.KW['max_iters']):.3f}; iteration counts differ on {bad.size}", flush=True)
    for j in bad[:4]:
        print(f"   target {j}: it gpu {it[j]} oracle {rit[j]}; err gpu {e[:, j]} oracle {re[:, j]}", flush=True)
