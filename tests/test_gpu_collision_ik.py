"""Collision-aware (bistage) IK: ``inverse_kinematics!(m, link, joints, target, sscc, sdf; use_bistage)``
(src/inverse_kinematics.jl:1-21) in the fridge scene of test/test_inverse_kinematics.jl:52-86.

The reference's own test solves PR2 (a network-downloaded robot) and builds its checker with an
un-iterated generator (:63), i.e. with no spheres.  Here: Fetch with the build-defined arm spheres (so
the constraint is live), the same fridge (door 2.0 rad, base (1.2, 0, 0)), targets inside the fridge's
open upper compartment.  Acceptance as the reference's: status :FTOL_REACHED, |dp| < 1e-3 and
|d RotZYX| < 1e-3, and every sphere distance >= margin (0.02) - 1e-6 (the reference's constraint is
dist - margin >= -1e-8 up to SLSQP's feasibility tolerance).  Sphere placement is parity-unpinned."""
import numpy as np
import pytest
import torch

from conftest import ARM, golden

import kinhip

pytestmark = pytest.mark.gpu


def _scene(with_base=False):
    m = kinhip.parse_urdf(golden("fetch.urdf"), with_base=with_base)
    fr = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
    sdf = kinhip.fridge_sdf(fr)
    sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
    return m, [m.find_joint(n) for n in ARM], sscc, sdf


def _pose(t, yaw=0.0):
    T = np.eye(4)
    c, s = np.cos(yaw), np.sin(yaw)
    T[:3, :3] = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
    T[:3, 3] = t
    return T


def _ypr(T):
    r = kinhip.rpy(T)
    return np.array([r[2], r[1], r[0]])


@pytest.mark.parametrize("target", [(1.0, 0.0, 1.25), (0.98, 0.08, 1.2), (0.95, -0.1, 1.3)])
def test_bistage_ik_in_fridge(target):
    m, arm, sscc, sdf = _scene()
    gl = m.find_link("gripper_link")
    T = _pose(target)
    # stage 1 alone (the collision-free problem) for the record
    m.set_joint_angles(arm, np.zeros(8))
    q1, st1 = kinhip.inverse_kinematics_(m, gl, arm, T, with_rot=True)
    d1 = kinhip.compute_coll_dists(sscc, arm, sdf)
    m.set_joint_angles(arm, np.zeros(8))
    q, status = kinhip.inverse_kinematics_(m, gl, arm, T, sscc, sdf, use_bistage=True, with_rot=True)
    d = kinhip.compute_coll_dists(sscc, arm, sdf)
    Tn = kinhip.get_transform(m, gl)
    print(f"target {target}: stage 1 {st1} min dist {d1.min():.4f}; bistage {status} min dist {d.min():.4f}, "
          f"|dp| {np.linalg.norm(Tn[:3, 3] - T[:3, 3]):.2e}")
    assert status == ":FTOL_REACHED"
    assert np.linalg.norm(Tn[:3, 3] - T[:3, 3]) < 1e-3
    assert np.linalg.norm(_ypr(Tn) - _ypr(T)) < 1e-3
    assert np.all(d >= 0.02 - 1e-6), d.min()
    lo = np.array([j.lower_limit for j in arm])
    hi = np.array([j.upper_limit for j in arm])
    assert np.all(q >= lo - 1e-9) and np.all(q <= hi + 1e-9)


@pytest.mark.parametrize("target,link,size", [((0.75, 0.15, 1.0), "elbow_flex_link", 0.08),
                                              ((0.7, -0.2, 1.1), "elbow_flex_link", 0.08),
                                              ((0.8, 0.0, 1.2), "upperarm_roll_link", 0.08),
                                              ((0.6, 0.3, 0.9), "forearm_roll_link", 0.06)])
def test_bistage_ik_moves_the_arm_off_an_obstacle(target, link, size):
    """A box pillar placed on `link` of the collision-free solution (stage 1 then collides for sure):
    stage 2 keeps the pose and moves the arm to the margin.  (Pillars where no nearby collision-free
    solution exists end in a constrained local minimum, as NLopt's SLSQP would; tools/cik_probe.py.)"""
    m, arm, sscc, sdf0 = _scene()
    gl = m.find_link("gripper_link")
    T = _pose(target)
    m.set_joint_angles(arm, np.zeros(8))
    kinhip.inverse_kinematics_(m, gl, arm, T)
    sdf = kinhip.UnionSDF(sdf0.sdfs + [kinhip.BoxSDF(_pose(kinhip.get_transform(m, m.find_link(link))[:3, 3]),
                                                     (size, size, size))])
    d1 = kinhip.compute_coll_dists(sscc, arm, sdf)
    assert d1.min() < 0  # the stage-1 solution is in collision
    m.set_joint_angles(arm, np.zeros(8))
    q, status = kinhip.inverse_kinematics_(m, gl, arm, T, sscc, sdf, use_bistage=True)
    d = kinhip.compute_coll_dists(sscc, arm, sdf)
    Tn = kinhip.get_transform(m, gl)
    assert status == ":FTOL_REACHED"
    assert np.linalg.norm(Tn[:3, 3] - T[:3, 3]) < 1e-3
    assert np.linalg.norm(_ypr(Tn) - _ypr(T)) < 1e-3
    assert np.all(d >= 0.02 - 1e-6), d.min()


def test_collision_ik_without_spheres_is_the_plain_problem():
    """test/test_inverse_kinematics.jl:63's checker has no spheres: no constraints, the pose problem."""
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    fr = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
    sdf = kinhip.fridge_sdf(fr)
    sscc = kinhip.SweptSphereCollisionChecker(m)
    T = _pose((0.3, -0.4, 1.2))
    gl = m.find_link("gripper_link")
    q, status = kinhip.inverse_kinematics_(m, gl, arm, T, sscc, sdf, use_bistage=False)
    assert status == ":FTOL_REACHED"
    Tn = kinhip.get_transform(m, gl)
    assert np.linalg.norm(Tn[:3, 3] - T[:3, 3]) < 1e-3
    assert np.linalg.norm(_ypr(Tn) - _ypr(T)) < 1e-3


def test_collision_ik_argument_errors():
    m, arm, sscc, sdf = _scene()
    with pytest.raises(TypeError):
        kinhip.inverse_kinematics_(m, m.find_link("gripper_link"), arm, np.eye(4), sscc, None)


def _oracle_scene(sdf):
    import oracle as O
    tree = O.parse_urdf_tree(golden("fetch.urdf"))
    om = O.OracleMech(tree)
    sph, rad, par = [], [], []
    for name, c, r in kinhip.FETCH_ARM_SPHERES:
        T = np.eye(4)
        T[:3, 3] = c
        sph.append(om.add_new_link(tree.link_id(name), T))
        rad.append(r)
        par.append(tree.link_id(name))
    box = O.OracleUnionSDF([b.pose for b in sdf.sdfs], [b.width for b in sdf.sdfs])
    _oracle_scene.parents = par
    return O, tree, om, sph, rad, box


def _check_batch(sdf, tg, Q, it, err, max_iters, dtype, min_conv):
    """Converged targets (iters <= max_iters) meet the reference's acceptance, recomputed by the oracle
    at the returned angles: |dp| < 1e-3, |d rpy| < 1e-3, every sphere >= margin - 1e-6 (fp32: 1e-5), within
    the joint limits."""
    O, tree, om, sph, rad, box = _oracle_scene(sdf)
    ids = [tree.joint_id(n) for n in ARM]
    gl = tree.link_id("gripper_link")
    conv = it.cpu().numpy() <= max_iters
    assert conv.mean() >= min_conv, conv.mean()
    q = Q.double().cpu().numpy()
    got = om.fk_batch(q, ids, [gl])[0]
    T = tg.double().cpu().numpy()
    dp = np.linalg.norm(got[9:] - T[9:], axis=0)
    assert np.all(dp[conv] < 1e-3), dp[conv].max()
    for k in np.nonzero(conv)[0][:: max(1, conv.sum() // 512)]:  # rpy on a sample (host loop)
        Ta, Tt = np.eye(4), np.eye(4)
        Ta[:3, :4] = got[:, k].reshape(4, 3).T
        Tt[:3, :4] = T[:, k].reshape(4, 3).T
        d = O.rpy(Ta) - O.rpy(Tt)
        assert np.all(np.abs((d + np.pi) % (2 * np.pi) - np.pi) < 1e-3), (k, d)
    dist, _ = O.coll_batch(om, box, q, ids, sph, rad, with_grad=False)
    ftol = 1e-6 if dtype == torch.float64 else 1e-5
    assert np.all(dist[:, conv] >= 0.02 - ftol), dist[:, conv].min()
    np.testing.assert_allclose(err[2].double().cpu().numpy()[conv], dist.min(0)[conv], atol=1e-5)
    lo = np.nan_to_num(np.array([kinhip.parse_urdf(golden("fetch.urdf")).find_joint(n).lower_limit for n in ARM]),
                       neginf=-1e9)
    hi = np.nan_to_num(np.array([kinhip.parse_urdf(golden("fetch.urdf")).find_joint(n).upper_limit for n in ARM]),
                       posinf=1e9)
    tol = 1e-6 if dtype == torch.float32 else 0
    assert np.all(q >= lo[:, None] - tol) and np.all(q <= hi[:, None] + tol)
    return conv


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_batched_collision_ik_in_fridge(dtype):
    """the bistage solve of test_bistage_ik_in_fridge for 4,096 targets in one launch per
    stage (CollisionIKPlan.solve: kin_ik_dls_batch_from, then kin_ik_coll_batch), targets spread over
    the fridge's open upper compartment (x 0.9..1.05, y +-0.12, z 1.15..1.32, yaw +-0.3)."""
    m, arm, sscc, sdf = _scene()
    gl = m.find_link("gripper_link")
    dev = torch.device("cuda", 0)
    N = 4096
    rng = np.random.default_rng(17)
    tg = np.zeros((12, N))
    for k in range(N):
        T = _pose((rng.uniform(0.9, 1.05), rng.uniform(-0.12, 0.12), rng.uniform(1.15, 1.32)), rng.uniform(-0.3, 0.3))
        tg[:, k] = np.concatenate([T[:3, :3].T.reshape(-1), T[:3, 3]])
    tg = torch.tensor(tg, dtype=dtype, device=dev).contiguous()
    plan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=dtype).specialize()
    Q0 = torch.zeros((8, N), dtype=dtype, device=dev)
    Q, it, err = plan.solve(sdf, tg, Q0, max_iters=128, restarts=3, seed=1)
    conv = _check_batch(sdf, tg, Q, it, err, 128, dtype, 0.9)
    # stage 1 alone would collide for some of them: the constraint did work
    print(f"batched bistage in the fridge {dtype}: converged {conv.mean():.4f}")


@pytest.mark.parametrize("target,link,size", [((0.75, 0.15, 1.0), "elbow_flex_link", 0.08),
                                              ((0.7, -0.2, 1.1), "elbow_flex_link", 0.08),
                                              ((0.8, 0.0, 1.2), "upperarm_roll_link", 0.08),
                                              ((0.6, 0.3, 0.9), "forearm_roll_link", 0.06)])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_batched_collision_ik_pillar(target, link, size, dtype):
    """test_bistage_ik_moves_the_arm_off_an_obstacle as a batch: 4,096 targets jittered by +-5 mm around
    the case's target, the pillar on the stage-1 solution's link (so stage 1 collides for most of them);
    both stages for all of them in one launch each, and every converged solution is off the pillar
    at the pose."""
    m, arm, sscc, sdf0 = _scene()
    gl = m.find_link("gripper_link")
    T0 = _pose(target)
    m.set_joint_angles(arm, np.zeros(8))
    kinhip.inverse_kinematics_(m, gl, arm, T0)
    sdf = kinhip.UnionSDF(sdf0.sdfs + [kinhip.BoxSDF(_pose(kinhip.get_transform(m, m.find_link(link))[:3, 3]),
                                                     (size, size, size))])
    dev = torch.device("cuda", 0)
    N = 4096
    rng = np.random.default_rng(5)
    tg = np.zeros((12, N))
    for k in range(N):
        T = _pose(np.asarray(target) + rng.uniform(-0.005, 0.005, 3))
        tg[:, k] = np.concatenate([T[:3, :3].T.reshape(-1), T[:3, 3]])
    tg = torch.tensor(tg, dtype=dtype, device=dev).contiguous()
    plan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=dtype).specialize()
    Q0 = torch.zeros((8, N), dtype=dtype, device=dev)
    Q1 = torch.empty_like(Q0)
    plan.ik_dls(tg, Q1, Q0=Q0, max_iters=64, restarts=3, seed=1, with_rot=2)
    _, _, D1 = sscc.plan(arm, dtype=dtype).run(sdf, Q1, dists=False, min_dist=True)
    Q, it, err = plan.solve(sdf, tg, Q0, max_iters=128, restarts=3, seed=1)
    conv = _check_batch(sdf, tg, Q, it, err, 128, dtype, 0.99)
    print(f"pillar {target} {dtype}: stage-1 solutions under the margin {float((D1 < 0.02).float().mean()):.3f}, "
          f"bistage converged {conv.mean():.4f}")
    assert float((D1 < 0.02).float().mean()) > 0.4


@pytest.mark.parametrize("spec,lanes,restarts", [(False, 0, 2), (False, 4, 2), (False, 4, 3), (True, 0, 2),
                                                 (True, 1, 2), (True, 4, 2), (True, 16, 2), (True, 64, 2),
                                                 (True, 64, 3)])
def test_collision_ik_iterates_vs_oracle(spec, lanes, restarts):
    """kin_ik_coll_batch (fp64) vs its CPU restatement (oracle or_ik_coll_batch): from the same seeds
    (the GPU's stage-1 solutions of 512 fridge targets) the same iteration counts, angles within 1e-7,
    errors and minimum sphere distances within 1e-9 -- generic and plan-specialised kernels, every lane
    layout (restarts = 2: 3 attempts, so a 4-group layout idles one group from the start),
    the reference's rpy objective with restarts.  The generic kernel's four attempt groups (lanes = 4) are
    the round-3 configuration that faulted (profiles/r04_ikc_fault.txt): re-enabled once the out-of-line
    trig call returned by value, at restarts = 2 and 3."""
    import oracle as O
    m, arm, sscc, sdf = _scene()
    gl = m.find_link("gripper_link")
    dev = torch.device("cuda", 0)
    N = 512
    rng = np.random.default_rng(23)
    tg = np.zeros((12, N))
    for k in range(N):
        T = _pose((rng.uniform(0.9, 1.05), rng.uniform(-0.12, 0.12), rng.uniform(1.15, 1.32)), rng.uniform(-0.3, 0.3))
        tg[:, k] = np.concatenate([T[:3, :3].T.reshape(-1), T[:3, 3]])
    tgt = torch.tensor(tg, dtype=torch.float64, device=dev).contiguous()
    plan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=torch.float64)
    if spec:
        plan.specialize()
    Q0 = torch.zeros((8, N), dtype=torch.float64, device=dev)
    Q1 = torch.empty_like(Q0)
    plan.ik_dls(tgt, Q1, Q0=Q0, max_iters=64, restarts=3, seed=2, with_rot=2)  # stage 1 (seeds for both)
    kw = dict(margin=0.02, band=0.01, weight=1.0, feas=1e-6, max_iters=96, lam=1e-2, tol_pos=1e-4, tol_rot=1e-4,
              max_step=0.5, with_rot=2, restarts=restarts, seed=7)
    Q, it, err = plan.ik_coll(sdf, tgt, torch.empty_like(Q1), Q0=Q1, lanes=lanes, **kw)
    O_, tree, om, sph, rad, box = _oracle_scene(sdf)
    ids = [tree.joint_id(n) for n in ARM]
    rq, rit, rerr = O.ik_coll_batch(om, box, Q1.cpu().numpy(), ids, tree.link_id("gripper_link"), tg, sph, rad,
                                    sphere_parents=_oracle_scene.parents, **kw)
    it = it.cpu().numpy()
    assert (it <= 96).mean() > 0.8
    np.testing.assert_array_equal(it, rit)
    # converged targets: angles 1e-7, err rows 1e-9.  A target no attempt solves returns its lowest-merit
    # attempt; attempts that end in the same constrained minimum tie in merit to the last bits (restarts = 3:
    # one of 512 here), so there the merits agree to 1e-9 while the angles may be another tying attempt's
    conv = it <= 96
    q, e = Q.cpu().numpy(), err.cpu().numpy()
    np.testing.assert_allclose(q[:, conv], rq[:, conv], atol=1e-7)
    np.testing.assert_allclose(e[:, conv], rerr[:, conv], atol=1e-9)

    def merit(x):
        return x[0] ** 2 + x[1] ** 2 + np.maximum(kw["margin"] - x[2], 0.0) ** 2
    np.testing.assert_allclose(merit(e[:, ~conv]), merit(rerr[:, ~conv]), rtol=1e-9, atol=1e-12)
    assert (np.abs(q - rq).max(0) > 1e-7).sum() <= 2  # (the tie rule covers a handful of targets only)


@pytest.mark.parametrize("spec", [False, True])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_collision_ik_lanes_identical(spec, dtype):
    """kin_ik_coll_batch runs the restart attempts of a target side by side in 4 lane groups and shares its
    spheres out over 16 lanes per group (specialised kernels; auto for small batches, or forced: lanes = 4,
    16, 64) or runs everything in sequence on one lane (lanes = 1): the sphere rows enter the normal
    equations in the same order, so angles, iteration counts and errors are bit-identical -- out of place
    and in place, with 4 attempts (one per group) and 5 (group 0 runs attempts 0 and 4); the generic
    kernels (one lane per target, or four attempt groups for lanes = 4) give the same answers."""
    m, arm, sscc, sdf = _scene()
    gl = m.find_link("gripper_link")
    dev = torch.device("cuda", 0)
    N = 1500  # not a multiple of the wave's 16 lane groups
    rng = np.random.default_rng(29)
    tg = np.zeros((12, N))
    for k in range(N):
        T = _pose((rng.uniform(0.85, 1.1), rng.uniform(-0.15, 0.15), rng.uniform(1.1, 1.35)), rng.uniform(-0.4, 0.4))
        tg[:, k] = np.concatenate([T[:3, :3].T.reshape(-1), T[:3, 3]])
    tgt = torch.tensor(tg, dtype=dtype, device=dev).contiguous()
    plan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=dtype)
    if spec:
        plan.specialize()
    Q0 = torch.zeros((8, N), dtype=dtype, device=dev)
    Q1 = torch.empty_like(Q0)
    plan.ik_dls(tgt, Q1, Q0=Q0, max_iters=64, restarts=3, seed=2, with_rot=2)
    for restarts, max_iters in ((3, 96), (4, 100)):
        kw = dict(margin=0.02, band=0.01, max_iters=max_iters, tol_pos=1e-4, tol_rot=1e-4, with_rot=2,
                  restarts=restarts, seed=7)
        ref = plan.ik_coll(sdf, tgt, torch.empty_like(Q1), Q0=Q1, lanes=1, **kw)
        for lanes in (0, 4, 16, 64):
            got = plan.ik_coll(sdf, tgt, torch.empty_like(Q1), Q0=Q1, lanes=lanes, **kw)
            for a, b in zip(got, ref):
                assert torch.equal(a, b), (restarts, lanes)
        Qi = Q1.clone()
        got = plan.ik_coll(sdf, tgt, Qi, lanes=0, **kw)  # in place
        for a, b in zip(got, ref):
            assert torch.equal(a, b), (restarts, "in place")
        it = ref[1].cpu().numpy()
        # the case exercises the schedule: targets solved in attempt 0, in a restart, and not at all
        L = max_iters // (restarts + 1)
        assert (it <= L).any() and ((it > L) & (it <= max_iters)).any(), np.bincount(np.minimum(it, max_iters + 1))


def _merit(m, gl, arm, sscc, sdf, T, margin=0.02):
    Tn = kinhip.get_transform(m, gl)
    d = kinhip.compute_coll_dists(sscc, arm, sdf)
    dp = np.linalg.norm(Tn[:3, 3] - T[:3, 3])
    dr = _ypr(Tn) - _ypr(T)
    dr = (dr + np.pi) % (2 * np.pi) - np.pi
    return dp ** 2 + float(dr @ dr) + max(0.0, margin - d.min()) ** 2, dp, d.min()


def test_infeasible_target_returns_the_best_attempt_vs_slsqp():
    """a pose the constraint forbids (an 8 cm box around the gripper's target point): the DLS
    stage 2 reports :MAXEVAL_REACHED with its best attempt -- not the last restart's end state -- and that
    answer's merit (pose error^2 + margin violation^2, what the kernel ranks attempts by) is no worse than
    what SciPy's SLSQP (the reference's solver family, constraint enforced) reaches from the same stage-1
    seed, up to a small slack; the SLSQP path itself ends feasible."""
    m, arm, sscc, sdf0 = _scene()
    gl = m.find_link("gripper_link")
    T = _pose((0.75, 0.15, 1.0))
    sdf = kinhip.UnionSDF(sdf0.sdfs + [kinhip.BoxSDF(_pose((0.75, 0.15, 1.0)), (0.08, 0.08, 0.08))])
    m.set_joint_angles(arm, np.zeros(8))
    q, status = kinhip.inverse_kinematics_(m, gl, arm, T, sscc, sdf, use_bistage=True)
    f_dls, dp_dls, dmin_dls = _merit(m, gl, arm, sscc, sdf, T)
    m.set_joint_angles(arm, np.zeros(8))
    q2, st2 = kinhip.inverse_kinematics_(m, gl, arm, T, sscc, sdf, use_bistage=True, solver="SLSQP")
    f_sq, dp_sq, dmin_sq = _merit(m, gl, arm, sscc, sdf, T)
    print(f"DLS {status}: merit {f_dls:.3e} |dp| {dp_dls:.3e} min d {dmin_dls:.4f}; "
          f"SLSQP {st2}: merit {f_sq:.3e} |dp| {dp_sq:.3e} min d {dmin_sq:.4f}")
    assert status == ":MAXEVAL_REACHED"
    assert np.all(np.isfinite(q))
    assert f_dls <= 1.5 * f_sq + 1e-4, (f_dls, f_sq)
    assert dmin_sq >= 0.02 - 1e-4  # SLSQP keeps the constraint (to its feasibility tolerance)


def test_slsqp_stage2_pose_accuracy_at_ftol():
    """the SLSQP stage 2 takes ftol as SciPy's ftol (the reference's ftol_abs = 1e-5 on
    f = |residual|^2): on a feasible target the pose still ends within the reference test's 1e-3."""
    m, arm, sscc, sdf = _scene()
    gl = m.find_link("gripper_link")
    T = _pose((1.0, 0.0, 1.25))
    m.set_joint_angles(arm, np.zeros(8))
    q, status = kinhip.inverse_kinematics_(m, gl, arm, T, sscc, sdf, use_bistage=True, solver="SLSQP")
    Tn = kinhip.get_transform(m, gl)
    d = kinhip.compute_coll_dists(sscc, arm, sdf)
    print(f"SLSQP {status}: |dp| {np.linalg.norm(Tn[:3, 3] - T[:3, 3]):.2e} min d {d.min():.4f}")
    assert status == ":FTOL_REACHED"
    assert np.linalg.norm(Tn[:3, 3] - T[:3, 3]) < 1e-3
    assert np.linalg.norm(_ypr(Tn) - _ypr(T)) < 1e-3
    assert d.min() >= 0.02 - 1e-4
