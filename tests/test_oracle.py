"""CPU oracle pinned against the reference's own fixtures and tests (no GPU).

Ports of the reference's test logic onto the C restatement:
  test/test_kinematics.jl:1-41   FK vs data/ground_truth.json (PR2), with/without base, twice (cache)
  test/test_kinematics.jl:43-73  analytic vs forward-difference Jacobian (eps 1e-7, atol 1e-5), rpy rows
  test/test_mechanism.jl:1-68    tree / rptable facts (Fetch; PR2 facts through the fragment)
  test/test_inverse_kinematics.jl:1-25  IK acceptance (|dp|, |drpy| <= 1e-3) -- DLS restatement
plus an independent numpy formulation and the committed golden fixture.
"""
import json

import numpy as np
import pytest

import numpy_ref as R
import oracle as O
from conftest import ARM, golden


@pytest.fixture(scope="module")
def gt():
    with open(golden("ground_truth.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def pr2():
    return O.parse_urdf_tree(golden("pr2_torso_rarm.urdf"))


@pytest.fixture(scope="module")
def fetch():
    return O.parse_urdf_tree(golden("fetch.urdf"))


def _rotz(t):
    return np.array([[np.cos(t), -np.sin(t), 0], [np.sin(t), np.cos(t), 0], [0, 0, 1]])


@pytest.mark.parametrize("with_base", [False, True])
def test_ground_truth_fk(gt, pr2, with_base):
    m = O.OracleMech(pr2, with_base=with_base)
    jids = [pr2.joint_id(n) for n in gt["joint_names"]]
    angles = list(gt["angle_vector"]) + ([0.3, 0.3, 0.3] if with_base else [])
    m.set_joint_angles(jids, angles)
    for _ in range(2):  # twice: cached values must equal fresh ones (test_kinematics.jl:21)
        for ln, pg in zip(gt["link_names"], gt["pose_list"]):
            T = m.get_transform(pr2.link_id(ln))
            pg = np.asarray(pg)
            r = O.rpy(T)
            ypr = np.array([r[2], r[1], r[0]])
            if with_base:
                np.testing.assert_allclose(T[:3, 3], _rotz(0.3) @ pg[:3] + [0.3, 0.3, 0], atol=1e-12)
                np.testing.assert_allclose(ypr, pg[3:] + [0.3, 0, 0], atol=1e-12)
            else:
                np.testing.assert_allclose(T[:3, 3], pg[:3], atol=1e-12)
                np.testing.assert_allclose(ypr, pg[3:], atol=1e-12)


@pytest.mark.parametrize("with_base", [False, True])
def test_pr2_two_arms_fixture_ground_truth(gt, with_base):
    """tests/golden/pr2_two_arms.urdf (the two-arm PR2 of the round-5 collision-IK tests) carries the chain
    data/ground_truth.json pins: its link poses at the fixture's angles equal the reference's to 1e-12, and
    the mirrored left arm is the right arm reflected in the x-z plane (y -> -y) at mirrored angles."""
    t = O.parse_urdf_tree(golden("pr2_two_arms.urdf"))
    m = O.OracleMech(t, with_base=with_base)
    jids = [t.joint_id(n) for n in gt["joint_names"]]
    base = [0.3, 0.3, 0.3] if with_base else []
    m.set_joint_angles(jids, list(gt["angle_vector"]) + base)
    for ln, pg in zip(gt["link_names"], gt["pose_list"]):
        T = m.get_transform(t.link_id(ln))
        pg = np.asarray(pg)
        if with_base:
            np.testing.assert_allclose(T[:3, 3], _rotz(0.3) @ pg[:3] + [0.3, 0.3, 0], atol=1e-12)
        else:
            np.testing.assert_allclose(T[:3, 3], pg[:3], atol=1e-12)
    # mirror: pan / roll joints (axes z, x) flip sign, the lift / flex joints (axis y) keep theirs
    m2 = O.OracleMech(t)
    rng = np.random.default_rng(3)
    names = ["shoulder_pan_joint", "shoulder_lift_joint", "upper_arm_roll_joint", "elbow_flex_joint",
             "forearm_roll_joint", "wrist_flex_joint", "wrist_roll_joint"]
    sign = np.array([-1, 1, -1, 1, -1, 1, -1.0])
    for _ in range(5):
        q = rng.uniform(-1, 0, 7)
        m2.set_joint_angles([t.joint_id("r_" + n) for n in names] + [t.joint_id("l_" + n) for n in names],
                            list(q) + list(sign * q))
        Tr = m2.get_transform(t.link_id("r_gripper_tool_frame"))
        Tl = m2.get_transform(t.link_id("l_gripper_tool_frame"))
        np.testing.assert_allclose(Tl[:3, 3], Tr[:3, 3] * [1, -1, 1], atol=1e-12)


@pytest.mark.parametrize("with_base", [False, True])
def test_fd_jacobian_all_links(gt, pr2, with_base):
    """test/test_kinematics.jl:43-73, every link, fixture angles and zeros."""
    m = O.OracleMech(pr2, with_base=with_base)
    jids = [pr2.joint_id(n) for n in gt["joint_names"]]
    a1 = np.array(list(gt["angle_vector"]) + ([0.3, 0.3, 0.3] if with_base else []))
    eps = 1e-7
    for angles in (a1, a1 * 0):
        for lid in range(1, len(pr2.link_names) + 1):
            m.set_joint_angles(jids, angles)
            Ja = m.get_jacobian(lid, jids, with_rot=True, rpy_jac=True)
            T0 = m.get_transform(lid)
            Jn = np.zeros_like(Ja)
            for i in range(len(angles)):
                a = angles.copy()
                a[i] += eps
                m.set_joint_angles(jids, a)
                T1 = m.get_transform(lid)
                Jn[:3, i] = (T1[:3, 3] - T0[:3, 3]) / eps
                Jn[3:, i] = (O.rpy(T1) - O.rpy(T0)) / eps
            np.testing.assert_allclose(Jn[:3], Ja[:3], atol=1e-5)
            if np.linalg.norm(Jn[3:, -3:]) < 1e4:
                np.testing.assert_allclose(Jn[3:], Ja[3:], atol=1e-5)


def test_fetch_mechanism_facts(fetch):
    """test/test_mechanism.jl:3-29, 54-67 on the oracle tree."""
    t = fetch
    base = t.link_id("base_link")
    kids = {t.link_names[t.joint_clink[j] - 1] for j in range(len(t.joint_names)) if t.joint_plink[j] == base}
    assert kids == {"r_wheel_link", "l_wheel_link", "torso_lift_link", "estop_link", "laser_link", "torso_fixed_link"}
    assert base not in set(t.joint_clink)
    sp = t.link_id("shoulder_pan_link")
    pj = [j for j in range(len(t.joint_names)) if t.joint_clink[j] == sp]
    assert t.joint_names[pj[0]] == "shoulder_pan_joint"
    assert t.link_names[t.joint_plink[pj[0]] - 1] == "torso_lift_link"
    for leaf in ["r_wheel_link", "l_wheel_link", "r_gripper_finger_link", "l_gripper_finger_link", "bellows_link2",
                 "estop_link", "laser_link", "torso_fixed_link", "head_camera_rgb_optical_frame",
                 "head_camera_depth_optical_frame"]:
        assert t.link_id(leaf) not in set(t.joint_plink)
    m = O.OracleMech(t)
    jid = t.joint_id
    assert m.is_relevant(jid("torso_lift_joint"), t.link_id("torso_lift_link"))
    assert m.is_relevant(jid("shoulder_pan_joint"), t.link_id("wrist_roll_link"))
    assert not m.is_relevant(jid("shoulder_pan_joint"), base)
    new = m.add_new_link(t.link_id("wrist_roll_link"), np.eye(4))
    assert new == len(t.link_names) + 1
    assert m.is_relevant(jid("torso_lift_joint"), new)


def test_pr2_fragment_rptable(pr2):
    m = O.OracleMech(pr2)
    assert m.is_relevant(pr2.joint_id("torso_lift_joint"), pr2.link_id("torso_lift_link"))
    assert not m.is_relevant(pr2.joint_id("r_wrist_flex_joint"), pr2.link_id("r_elbow_flex_link"))


def test_oracle_vs_numpy(fetch):
    ids = [fetch.joint_id(n) for n in ARM]
    rng = np.random.default_rng(1)
    for wb in (False, True):
        q = rng.uniform(-2, 2, (len(ids) + (3 if wb else 0), 300))
        m = O.OracleMech(fetch, with_base=wb)
        gl = fetch.link_id("gripper_link")
        for rpyj in (False, True):
            pose, jac = m.fk_jac_batch(q, ids, gl, ids, True, rpyj)
            T, Jm = R.jacobian(fetch, q, ids, gl, ids, True, rpyj, wb)
            np.testing.assert_allclose(pose, R.pose12(T), atol=1e-12)
            np.testing.assert_allclose(jac, Jm.transpose(2, 1, 0), atol=1e-11)


def test_golden_fixture_reproduced(fetch):
    g = np.load(golden("fetch_fk_jac_golden.npz"))
    ids = [fetch.joint_id(n) for n in g["joint_names"]]
    m = O.OracleMech(fetch)
    poses = m.fk_batch(g["q"], ids, list(range(1, len(fetch.link_names) + 1)))
    np.testing.assert_array_equal(poses, g["poses"])
    gl = fetch.link_id("gripper_link")
    _, jg = m.fk_jac_batch(g["q"], ids, gl, ids, True, False)
    np.testing.assert_array_equal(jg, g["jac_geo"])
    # sanity derived in SURVEY.md 8c(5): gripper_link at q = 0
    m0 = O.OracleMech(fetch)
    np.testing.assert_allclose(m0.get_transform(gl)[:3, 3], [1.1281, 0, 0.78601], atol=1e-12)


def test_get_jacobian_bang_leaves_untouched(fetch):
    """get_jacobian! writes only relevant columns (src/algorithm.jl:91-96)."""
    m = O.OracleMech(fetch)
    ids = [fetch.joint_id(n) for n in ARM] + [fetch.joint_id("head_pan_joint")]
    buf = np.full((6, len(ids)), 7.0)
    J = m.get_jacobian(fetch.link_id("gripper_link"), ids, True, False, mat=buf)
    assert np.all(J[:, -1] == 7.0)               # head_pan irrelevant to the gripper
    assert np.all(J[3:, 0] == 7.0)               # torso is prismatic: rows 4:6 untouched
    with pytest.raises(ValueError):              # relevant fixed joint -> MethodError
        m.get_jacobian(fetch.link_id("gripper_link"), [fetch.joint_id("gripper_axis")], True)


def test_ik_dls_oracle_reference_target(fetch):
    """test/test_inverse_kinematics.jl:1-25 acceptance, via the build-defined DLS."""
    ids = [fetch.joint_id(n) for n in ARM]
    gl = fetch.link_id("gripper_link")
    m = O.OracleMech(fetch)
    T = np.eye(4)
    T[:3, 3] = [0.3, -0.4, 1.2]
    tgt = T[:3, :4].T.reshape(12, 1)
    q, it, err = m.ik_dls_batch(np.zeros((8, 1)), ids, gl, tgt, max_iters=200, tol_pos=1e-4, tol_rot=1e-4)
    assert it[0] < 200
    m.set_joint_angles(ids, q[:, 0])
    Tn = m.get_transform(gl)
    np.testing.assert_allclose(Tn[:3, 3], T[:3, 3], atol=1e-3)
    np.testing.assert_allclose(O.rpy(Tn), O.rpy(T), atol=1e-3)


def test_nakamura_oracle_reaches_point(fetch):
    ids = [fetch.joint_id(n) for n in ARM]
    gl = fetch.link_id("gripper_link")
    m = O.OracleMech(fetch)
    target = np.array([0.7, 0.2, 0.9])
    q = m.point_ik_nakamura(gl, ids, target)
    m.set_joint_angles(ids, q)
    assert np.linalg.norm(m.get_transform(gl)[:3, 3] - target) < 1e-3


def test_ik_objective_gradient(fetch):
    """f_objective (src/inverse_kinematics.jl:38-50): grad = -2 J_rpy^T diff vs finite differences."""
    ids = [fetch.joint_id(n) for n in ARM]
    gl = fetch.link_id("gripper_link")
    m = O.OracleMech(fetch)
    T = np.eye(4)
    T[:3, 3] = [0.5, -0.2, 1.0]
    a = np.array([0.1, 0.2, -0.3, 0.4, 0.5, -0.6, 0.3, 0.2])
    f0, g = m.ik_objective(gl, ids, T, a)
    eps = 1e-7
    for i in range(8):
        b = a.copy()
        b[i] += eps
        f1, _ = m.ik_objective(gl, ids, T, b)
        assert abs((f1 - f0) / eps - g[i]) < 1e-4


def _axis_angle(u, th):
    u = np.asarray(u, np.float64) / np.linalg.norm(u)
    K = np.array([[0, -u[2], u[1]], [u[2], 0, -u[0]], [-u[1], u[0], 0]])
    T = np.eye(4)
    T[:3, :3] = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    return T


@pytest.mark.parametrize("u", [(1, 1, 0), (1, 0, 0), (0, 1, 1), (1, 2, 3), (-2, 1, 0.5)])
def test_rot_error_pi_branch(u):
    """The IK's rotation error at a pi rotation (sin ~ 0, cos < 0 branch) returns pi * u for a
    rotation about any axis, not only coordinate axes (E = 2uu^T - I: off-diagonals are 2 u_k u_b)."""
    R0 = _axis_angle((0.3, -0.2, 0.9), 0.7)
    Rt = _axis_angle(u, np.pi) @ R0  # target = Rot(u, pi) * current
    w = O.rot_error(Rt, R0)
    un = np.asarray(u, np.float64) / np.linalg.norm(u)
    ok = min(np.abs(w - np.pi * un).max(), np.abs(w + np.pi * un).max())  # +-u is the same rotation
    assert ok < 1e-6, (w, np.pi * un)


def test_rot_error_generic_angles():
    R0 = _axis_angle((0.1, 0.5, -0.4), 1.1)
    for th in (1e-3, 0.5, 2.0, 3.1):
        u = np.array([0.2, -0.7, 0.4])
        w = O.rot_error(_axis_angle(u, th) @ R0, R0)
        np.testing.assert_allclose(w, th * u / np.linalg.norm(u), atol=1e-9)


def test_ik_iters_contract(fetch):
    """kinhip.h: iters <= max_iters iff converged; a target that converges at exactly max_iters reports
    max_iters, a failure max_iters + 1."""
    ids = [fetch.joint_id(n) for n in ARM]
    gl = fetch.link_id("gripper_link")
    m = O.OracleMech(fetch)
    T = np.eye(4)
    T[:3, 3] = [0.3, -0.4, 1.2]
    tgt = T[:3, :4].T.reshape(12, 1)
    q, it, err = m.ik_dls_batch(np.zeros((8, 1)), ids, gl, tgt, max_iters=200, tol_pos=1e-4, tol_rot=1e-4)
    k = int(it[0])
    assert k <= 200 and err[0, 0] < 1e-4
    _, it2, err2 = m.ik_dls_batch(np.zeros((8, 1)), ids, gl, tgt, max_iters=k, tol_pos=1e-4, tol_rot=1e-4)
    assert int(it2[0]) == k and err2[0, 0] < 1e-4  # converged exactly at max_iters
    _, it3, err3 = m.ik_dls_batch(np.zeros((8, 1)), ids, gl, tgt, max_iters=k - 1, tol_pos=1e-4, tol_rot=1e-4)
    assert int(it3[0]) == k  # (k - 1) + 1: not converged
    assert not (err3[0, 0] < 1e-4 and err3[1, 0] < 1e-4)


@pytest.mark.parametrize("damp_err", [0.0, 0.01, 0.3])
def test_ik_damped_step_restated(fetch, damp_err):
    """One step of the oracle's DLS IK (or_ik_dls_batch) against its statement written out in numpy:
    dq = J^T (J J^T + (lambda^2 + damp_err (|dp|^2 + |rot|^2)) I)^-1 e with e = [p* - p; log(R* R^T)],
    |dq|_inf clamped to max_step, q clamped to the limits -- the error-scaled damping of
    kin_ik_params.damp_err included (from inside the limits: no joint is held)."""
    m = O.OracleMech(fetch)
    ids = [fetch.joint_id(n) for n in ARM]
    gl = fetch.link_id("gripper_link")
    rng = np.random.default_rng(3)
    lo = np.array([fetch.joint_lower[j - 1] for j in ids], dtype=float)
    hi = np.array([fetch.joint_upper[j - 1] for j in ids], dtype=float)
    lo = np.where(np.isfinite(lo), lo, -np.pi)
    hi = np.where(np.isfinite(hi), hi, np.pi)
    N = 16
    q0 = lo[:, None] + (hi - lo)[:, None] * (0.25 + 0.5 * rng.random((8, N)))
    qt = lo[:, None] + (hi - lo)[:, None] * (0.25 + 0.5 * rng.random((8, N)))
    tgt = m.fk_batch(qt, ids, [gl])[0]
    lam, ms = 1e-2, 0.5
    q1, _, _ = m.ik_dls_batch(q0, ids, gl, tgt, max_iters=1, lam=lam, max_step=ms, tol_pos=0.0, tol_rot=0.0,
                              damp_err=damp_err)
    pose, J = m.fk_jac_batch(q0, ids, gl, ids)
    for i in range(N):
        T = np.eye(4)
        T[:3, :4] = tgt[:, i].reshape(4, 3).T
        Tn = np.eye(4)
        Tn[:3, :4] = pose[:, i].reshape(4, 3).T
        e = np.concatenate([T[:3, 3] - Tn[:3, 3], O.rot_error(T, Tn)])
        Ji = J[:, :, i].T  # [6, 8]
        l2 = lam * lam + damp_err * (e[:3] @ e[:3] + e[3:] @ e[3:])
        dq = Ji.T @ np.linalg.solve(Ji @ Ji.T + l2 * np.eye(6), e)
        sc = min(1.0, ms / np.abs(dq).max())
        ref = np.clip(q0[:, i] + sc * dq, lo, hi)
        np.testing.assert_allclose(q1[:, i], ref, atol=1e-12)
