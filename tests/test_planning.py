"""Planning constraints over waypoints (src/planning.jl).

CPU: the host assemblies (Objective, ConfigurationConstraint, EqConst, create_straight_trajectory)
against direct restatements of src/planning.jl.
GPU: IneqConst / PoseConstraint (one batched launch over all waypoints) against the oracle's
restatement (oracle.ineq_const / oracle.pose_const), and the reference's planning test
(test/test_planning.jl) end to end with SLSQP on the host.  The spheres are build-defined
(kinhip.FETCH_LINK_SPHERES; mesh-derived spheres are offline-unavailable): parity unpinned for
sphere placement, pinned for the constraint arithmetic.
"""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import ARM, golden


def test_objective_second_differences():
    import kinhip
    rng = np.random.default_rng(0)
    n_wp, w = 7, np.array([1.0, 2.0, 0.5])
    F = kinhip.Objective(n_wp, w)
    xi = rng.standard_normal(n_wp * 3)
    X = xi.reshape(n_wp, 3)
    ref = sum(float(np.sum(w ** 2 * (X[i - 1] - 2 * X[i] + X[i + 1]) ** 2)) for i in range(1, n_wp - 1))
    g = np.zeros(xi.size)
    assert abs(F(xi, g) - ref) < 1e-10
    eps = 1e-6
    fd = np.array([(F(xi + eps * e) - F(xi - eps * e)) / (2 * eps) for e in np.eye(xi.size)])
    np.testing.assert_allclose(g, fd, atol=1e-6)


def test_straight_trajectory_and_eq_layout():
    import kinhip
    xi = kinhip.create_straight_trajectory([0.0, 1.0], [1.0, 3.0], 5)
    np.testing.assert_allclose(xi.reshape(5, 2), [[0, 1], [0.25, 1.5], [0.5, 2], [0.75, 2.5], [1, 3]])
    c1 = kinhip.ConfigurationConstraint(1, 2, [0.0, 1.0])
    c2 = kinhip.ConfigurationConstraint(5, 2, [1.0, 3.0])
    H = kinhip.EqConst(5, [c1, c2])
    x = xi + 0.1
    H(x, H.val_vec, H.jac_mat)
    np.testing.assert_allclose(H.val_vec, [-0.1, -0.1, -0.1, -0.1])
    assert H.jac_mat.shape == (10, 4)
    np.testing.assert_allclose(H.jac_mat[0:2, 0:2], -np.eye(2))
    np.testing.assert_allclose(H.jac_mat[8:10, 2:4], -np.eye(2))
    assert np.count_nonzero(H.jac_mat) == 4


def _T(t):
    T = np.eye(4)
    T[:3, 3] = t
    return T


COLL_LINKS = ["wrist_flex_link", "torso_lift_link", "upperarm_roll_link", "elbow_flex_link"]  # test_planning.jl:17-20


def _setup(with_base):
    import kinhip
    m = kinhip.parse_urdf(golden("fetch.urdf"), with_base=with_base)
    joints = [m.find_joint(n) for n in ARM]
    sscc = kinhip.SweptSphereCollisionChecker(m)
    for n in COLL_LINKS:
        kinhip.add_coll_links(sscc, m.find_link(n))
    sdf = kinhip.UnionSDF([kinhip.BoxSDF(_T((0.4, -0.25, 0.7)), (0.05, 0.05, 0.5))])
    tree = O.parse_urdf_tree(golden("fetch.urdf"))
    om = O.OracleMech(tree, with_base=with_base)
    sph, rad = [], []
    for n in COLL_LINKS:
        for c, r in kinhip.FETCH_LINK_SPHERES[n]:
            sph.append(om.add_new_link(tree.link_id(n), _T(c)))
            rad.append(r)
    return m, joints, sscc, sdf, tree, om, sph, rad


@pytest.mark.gpu
@pytest.mark.parametrize("with_base", [False, True])
def test_gpu_ineq_const_vs_oracle(with_base):
    import kinhip
    m, joints, sscc, sdf, tree, om, sph, rad = _setup(with_base)
    n_wp, margin = 10, 0.03
    n_dof = 8 + (3 if with_base else 0)
    rng = np.random.default_rng(3)
    xi = rng.uniform(-1.2, 1.2, n_wp * n_dof) * 0.8
    G = kinhip.IneqConst(sscc, joints, sdf, n_wp, margin)
    assert (G.n_dof, G.n_coll, G.n_cons) == (n_dof, len(sph), len(sph) * n_wp)
    G(xi, G.val_vec, G.jac_mat)
    rv, rj = O.ineq_const(om, O.OracleUnionSDF([_T((0.4, -0.25, 0.7))], [[0.05, 0.05, 0.5]]), xi,
                          [tree.joint_id(n) for n in ARM], sph, rad, n_wp, margin)
    np.testing.assert_allclose(G.val_vec, rv, atol=1e-9)
    assert np.all(G.val_vec <= 0.05 + 1e-12)  # truncation at margin + 0.05, minus margin
    bad = np.abs(G.jac_mat - rj) > 2e-5  # analytic vs the reference's forward-difference SDF gradient
    assert bad.mean() < 1e-3
    # off-diagonal blocks untouched (zero)
    nd, nc = n_dof, len(sph)
    mask = np.zeros_like(rj, bool)
    for i in range(n_wp):
        mask[nd * i:nd * (i + 1), nc * i:nc * (i + 1)] = True
    assert not np.any(G.jac_mat[~mask])


@pytest.mark.gpu
def test_gpu_ineq_const_many_trajectories():
    """One launch over B trajectories x n_wp waypoints equals per-trajectory evaluation."""
    import kinhip
    m, joints, sscc, sdf, *_ = _setup(False)
    G = kinhip.IneqConst(sscc, joints, sdf, 10, 0.02)
    rng = np.random.default_rng(4)
    B = 64
    Q = torch.tensor(rng.uniform(-1, 1, (8, B * 10)), dtype=torch.float64, device="cuda")
    V, J = G.eval_batch(Q)
    for b in (0, 17, 63):
        xi = Q[:, b * 10:(b + 1) * 10].T.reshape(-1).cpu().numpy()
        G(xi, G.val_vec, G.jac_mat)
        np.testing.assert_array_equal(G.val_vec, V[:, b * 10:(b + 1) * 10].T.reshape(-1).cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("with_rot", [True, False])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_gpu_pose_const_vs_oracle(with_rot, dtype):
    import kinhip
    m, joints, sscc, sdf, tree, om, sph, rad = _setup(False)
    gl = m.find_link("gripper_link")
    target = np.eye(4)
    target[:3, :3] = O.rpy_to_matrix([0.3, -0.2, 0.5])
    target[:3, 3] = [0.3, -0.4, 1.2]
    pc = kinhip.PoseConstraint(3, 8, gl, target, with_rot, m, joints, dtype=dtype)
    rng = np.random.default_rng(5)
    tol = 1e-9 if dtype == torch.float64 else 3e-5
    for _ in range(3):
        q = rng.uniform(-1, 1, 8)
        val = np.zeros(pc.n_cons)
        jac = np.zeros((8 * 5, pc.n_cons))
        pc(q, val, jac)
        rv, rJ = O.pose_const(om, q, [tree.joint_id(n) for n in ARM], tree.link_id("gripper_link"), target, with_rot)
        np.testing.assert_allclose(val, rv, atol=tol)
        np.testing.assert_allclose(jac[16:24, :], rJ.T, atol=tol)  # waypoint 3 -> rows 16:24
        assert not np.any(jac[:16]) and not np.any(jac[24:])
    # batched form with per-configuration targets
    N = 1000
    Q = torch.tensor(rng.uniform(-1, 1, (8, N)), dtype=dtype, device="cuda")
    Qt = torch.tensor(rng.uniform(-1, 1, (8, N)), dtype=dtype, device="cuda")
    plan = m.plan(joints, out_links=[gl], dtype=dtype)
    tg = plan.run(Qt)[0][0].contiguous()
    V, J, P = pc.eval_batch(0, Q, tg)
    ids = [tree.joint_id(n) for n in ARM]
    qn, tn = Q.double().cpu().numpy(), Qt.double().cpu().numpy()
    for i in (0, 500, 999):
        Tt = np.eye(4)
        ptn, _ = om.fk_jac_batch(tn[:, i:i + 1], ids, tree.link_id("gripper_link"), ids)
        Tt[:3, :] = ptn[:, 0].reshape(4, 3).T
        rv, rJ = O.pose_const(om, qn[:, i], ids, tree.link_id("gripper_link"), Tt, with_rot)
        np.testing.assert_allclose(V[:, i].double().cpu().numpy(), rv, atol=tol * 10)
        np.testing.assert_allclose(J[:, :, i].double().cpu().numpy(), rJ.T, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("with_base", [False, True])
def test_gpu_plan_trajectory(with_base):
    """test/test_planning.jl: IK goal for (0.3, -0.4, 1.2) without rotation, 10 waypoints around a
    thin box; every waypoint clears the box by more than -1e-2."""
    import kinhip
    m, joints, sscc, sdf, *_ = _setup(with_base)
    q_start = m.get_joint_angles(joints)
    gl = m.find_link("gripper_link")
    q_goal, status = kinhip.inverse_kinematics_(m, gl, joints, _T((0.3, -0.4, 1.2)), with_rot=False)
    assert status == ":FTOL_REACHED"
    # The reference's goal is its SLSQP IK solution, collision-free for its mesh-derived spheres.
    # With the build-defined spheres take the first collision-free solution of a batched IK from
    # seeded random starts (the batched engine's own use case).
    n_dof = len(q_start)
    plan = m.plan(joints, out_links=[gl], jac_link=gl, jac_joints=joints, dtype=torch.float64)
    N = 256
    g = torch.Generator().manual_seed(11)
    Q0 = (torch.rand((n_dof, N), generator=g, dtype=torch.float64) * 2 - 1).cuda()
    if with_base:
        Q0[8:] = 0.0
    tgt = torch.tensor(np.repeat(_T((0.3, -0.4, 1.2))[:3, :4].T.reshape(12, 1), N, axis=1), device="cuda")
    Q, it, _ = plan.ik_dls(tgt, Q0.contiguous(), with_rot=False, max_iters=64)
    _, _, mn = sscc.plan(joints, dtype=torch.float64).run(sdf, Q, dists=False, min_dist=True)
    ok = ((it <= 64) & (mn > 0.05)).nonzero()
    assert ok.numel() > 0
    q_goal = Q[:, int(ok[0, 0])].cpu().numpy()
    q_seq, status = kinhip.plan_trajectory(sscc, joints, sdf, q_start, q_goal, 10, ftol_abs=1e-5)
    assert status == ":SUCCESS"
    np.testing.assert_allclose(q_seq[:, 0], q_start, atol=1e-6)
    np.testing.assert_allclose(q_seq[:, -1], q_goal, atol=1e-6)
    for i in range(10):
        m.set_joint_angles(joints, q_seq[:, i])
        assert np.all(kinhip.compute_coll_dists(sscc, joints, sdf) > -1e-2)


@pytest.mark.parametrize("solver", ["NLOPT", ":NLOPT", "IPOPT", "bogus"])
def test_plan_trajectory_refuses_unavailable_solvers(solver):
    """NLopt / Ipopt are not installed: the planner refuses them instead of relabelling SciPy."""
    import kinhip
    with pytest.raises(ValueError):
        kinhip.plan_trajectory(None, [], None, [], [], 10, solver=solver)
