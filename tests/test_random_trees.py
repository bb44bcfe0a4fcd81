"""Property tests on seeded random kinematic trees (long chains -> phase-A bounds 4..32, branches ->
phase-B LDS slots, every joint type, odd axes, static chains held at random angles, base or not).

CPU: the native URDF parser against the oracle's xml.etree reader.
GPU: FK of random link sets + the Jacobian of a random link over random joint columns (relevant or
not, in random order, repeated), every flag combination, vs the oracle in fp64 (1e-9) and fp32.
"""
import os

import numpy as np
import pytest
import torch

import oracle as O
from randtree import random_urdf

SEEDS = list(range(48))


def _write(tmp_path, text, k):
    p = os.path.join(tmp_path, f"rand{k}.urdf")
    with open(p, "w") as f:
        f.write(text)
    return p


@pytest.mark.parametrize("seed", SEEDS)
def test_native_parser_matches_oracle_reader(tmp_path, seed):
    import kinhip
    rng = np.random.default_rng(seed)
    p = _write(str(tmp_path), random_urdf(rng, int(rng.integers(2, 40))), seed)
    t = O.parse_urdf_tree(p)
    m = kinhip.parse_urdf(p)
    assert [l.name for l in m.links] == t.link_names
    assert [j.name for j in m.joints] == t.joint_names
    for k, j in enumerate(m.joints):
        assert j.plink_id == t.joint_plink[k] and j.clink_id == t.joint_clink[k]
        np.testing.assert_allclose(j.pose, t.joint_pose[k], atol=1e-14)
        if t.joint_type[k] != 0:
            np.testing.assert_allclose(j.axis, t.joint_axis[k], atol=1e-14)
        assert j.lower_limit == t.joint_lower[k] and j.upper_limit == t.joint_upper[k]
    for lid, (ext, org) in t.link_box.items():
        meta = m.links[lid - 1].geometric_meta_data
        np.testing.assert_allclose(meta.extents, ext, atol=1e-14)
        np.testing.assert_allclose(meta.origin, org, atol=1e-14)


def _case(rng, t):
    J = len(t.joint_names)
    moving = [k + 1 for k in range(J) if t.joint_type[k] != 0]
    fixed = [k + 1 for k in range(J) if t.joint_type[k] == 0]
    nq = int(rng.integers(1, min(len(moving), 12) + 1))
    q_ids = [int(x) for x in rng.choice(moving, nq, replace=False)]
    if fixed and rng.random() < 0.3:
        q_ids.insert(int(rng.integers(0, len(q_ids) + 1)), int(rng.choice(fixed)))  # ignored by joint_transform
    L = len(t.link_names)
    outs = [int(x) for x in rng.choice(np.arange(1, L + 1), int(rng.integers(1, min(L, 6) + 1)), replace=False)]
    jac_link = int(rng.integers(1, L + 1))
    jac_ids = [int(x) for x in rng.choice(moving, int(rng.integers(1, min(len(moving), 10) + 1)))]  # repeats ok
    return q_ids, outs, jac_link, jac_ids


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_gpu_random_tree_vs_oracle(tmp_path, seed):
    import kinhip
    from kinhip._lib import KinError, KIN_E_UNSUPPORTED
    rng = np.random.default_rng(1000 + seed)
    p = _write(str(tmp_path), random_urdf(rng, int(rng.integers(3, 40)), chain_bias=rng.uniform(0.5, 0.95)), seed)
    t = O.parse_urdf_tree(p)
    if not any(t.joint_type != 0):
        pytest.skip("no moving joint")
    with_base = bool(rng.random() < 0.4)
    m = kinhip.parse_urdf(p, with_base=with_base)
    om = O.OracleMech(t, with_base=with_base)
    q_ids, outs, jac_link, jac_ids = _case(rng, t)
    # joints outside the batch held at random angles (static chains baked into the plan)
    others = [k + 1 for k in range(len(t.joint_names)) if k + 1 not in q_ids]
    ang = rng.uniform(-1, 1, len(others))
    for jid, a in zip(others, ang):
        m.set_joint_angle(m.joints[jid - 1], float(a))
    om.set_joint_angles(others, np.concatenate([ang, np.zeros(3) if with_base else []]))
    with_rot, rpy_jac, zero_fill = bool(rng.random() < 0.7), bool(rng.random() < 0.4), bool(rng.random() < 0.5)
    N = int(rng.choice([1, 63, 257, 1000]))
    Q = rng.uniform(-2, 2, (len(q_ids) + (3 if with_base else 0), N))
    for k, jid in enumerate(q_ids):
        if t.joint_type[jid - 1] == 2:
            Q[k] *= 0.2
    qj = [m.joints[j - 1] for j in q_ids]
    for dtype, tol in ((torch.float64, 1e-9), (torch.float32, 3e-4)):
        try:
            plan = m.plan(qj, out_links=[m.links[o - 1] for o in outs], jac_link=m.links[jac_link - 1],
                          jac_joints=[m.joints[j - 1] for j in jac_ids], with_rot=with_rot, rpy_jac=rpy_jac,
                          zero_fill=zero_fill, dtype=dtype)
        except KinError as e:
            if e.code == KIN_E_UNSUPPORTED:
                pytest.skip(f"outside the engine limits: {e}")
            raise
        Qd = torch.tensor(Q, dtype=dtype, device="cuda")
        rows = 6 if with_rot else 3
        ncol = len(jac_ids) + (3 if with_base else 0)
        init = rng.uniform(-9, -8, (ncol, rows, N))  # sentinel: untouched entries must keep it
        Jd = torch.tensor(init, dtype=dtype, device="cuda")
        P, Jd = plan.run(Qd, jac=Jd)
        Qr = Qd.double().cpu().numpy()
        rp = om.fk_batch(Qr, q_ids, outs)
        np.testing.assert_allclose(P.double().cpu().numpy(), rp, atol=tol)
        _, rj = om.fk_jac_batch(Qr, q_ids, jac_link, jac_ids, with_rot, rpy_jac, zero_fill=zero_fill,
                                jac_init=init if dtype == torch.float64 else Jd.double().cpu().numpy() * 0 + init)
        got = Jd.double().cpu().numpy()
        if dtype == torch.float32:  # sentinel was rounded to fp32 on the device
            rj = np.where(rj == init, init.astype(np.float32).astype(np.float64), rj)
        np.testing.assert_allclose(got, rj, atol=tol, rtol=1e-4 if dtype == torch.float32 else 1e-9)
        if seed < 24:  # plan specialisation (constant-folded program) == generic kernel, bit for bit
            spe = m.plan(qj, out_links=[m.links[o - 1] for o in outs], jac_link=m.links[jac_link - 1],
                         jac_joints=[m.joints[j - 1] for j in jac_ids], with_rot=with_rot, rpy_jac=rpy_jac,
                         zero_fill=zero_fill, dtype=dtype).specialize(kinhip.KIN_SPEC_FK)
            P2, J2 = spe.run(Qd, jac=torch.tensor(init, dtype=dtype, device="cuda"))
            assert torch.equal(P2, P) and torch.equal(J2, Jd)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS[:24])
def test_gpu_random_tree_collision_vs_oracle(tmp_path, seed):
    """Spheres on random links of random trees (often several moving chains -> multi-program plans)
    against random boxes: distances, min distance and gradients vs the oracle (fp64)."""
    import kinhip
    from kinhip._lib import KinError, KIN_E_UNSUPPORTED
    rng = np.random.default_rng(5000 + seed)
    p = _write(str(tmp_path), random_urdf(rng, int(rng.integers(3, 30)), chain_bias=rng.uniform(0.4, 0.9)), seed)
    t = O.parse_urdf_tree(p)
    moving = [k + 1 for k in range(len(t.joint_names)) if t.joint_type[k] != 0]
    if not moving:
        pytest.skip("no moving joint")
    with_base = bool(rng.random() < 0.4)
    m = kinhip.parse_urdf(p, with_base=with_base)
    om = O.OracleMech(t, with_base=with_base)
    q_ids = [int(x) for x in rng.choice(moving, int(rng.integers(1, min(len(moving), 10) + 1)), replace=False)]
    sscc = kinhip.SweptSphereCollisionChecker(m)
    sph, rad = [], []
    for _ in range(int(rng.integers(1, 10))):
        lk = int(rng.integers(1, len(t.link_names) + 1))
        c, r = rng.uniform(-0.1, 0.1, 3), float(rng.uniform(0.02, 0.1))
        sscc.add_coll_sphere(m.links[lk - 1], c, r)
        T = np.eye(4)
        T[:3, 3] = c
        sph.append(om.add_new_link(lk, T))
        rad.append(r)
    poses, widths = [], []
    for _ in range(5):
        T = np.eye(4)
        if rng.random() < 0.5:
            T[:3, :3] = O.rpy_to_matrix(rng.uniform(-np.pi, np.pi, 3))
        T[:3, 3] = rng.uniform(-1, 1, 3)
        poses.append(T)
        widths.append(rng.uniform(0.05, 0.5, 3))
    sdf = kinhip.UnionSDF([kinhip.BoxSDF(P, w) for P, w in zip(poses, widths)])
    try:
        plan = sscc.plan([m.joints[j - 1] for j in q_ids], dtype=torch.float64)
    except KinError as e:
        if e.code == KIN_E_UNSUPPORTED:
            pytest.skip(f"outside the engine limits: {e}")
        raise
    N = 300
    Q = rng.uniform(-2, 2, (len(q_ids) + (3 if with_base else 0), N))
    Qd = torch.tensor(Q, dtype=torch.float64, device="cuda")
    D, G, Mn = plan.run(sdf, Qd, grads=True, min_dist=True)
    rd, rg = O.coll_batch(om, O.OracleUnionSDF(poses, widths), Q, q_ids, sph, rad)
    np.testing.assert_allclose(D.cpu().numpy(), rd, atol=1e-9)
    np.testing.assert_allclose(Mn.cpu().numpy(), rd.min(0), atol=1e-9)
    assert (np.abs(G.cpu().numpy() - rg) > 2e-5 * (1 + np.abs(rg))).mean() < 2e-3
    # specialised (chain + spheres folded; multi-chain plans specialise every program) == generic
    spe = sscc.plan([m.joints[j - 1] for j in q_ids], dtype=torch.float64).specialize()
    for x, y in zip((D, G, Mn), spe.run(sdf, Qd, grads=True, min_dist=True)):
        assert torch.equal(x, y)
