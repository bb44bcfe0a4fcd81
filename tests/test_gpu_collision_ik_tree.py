"""Collision-aware IK on the reference's scene shapes (/root/reference/fridge_demo.jl:13-37,
test/test_inverse_kinematics.jl:52-86): spheres on more than one moving chain, a planar base, and a union
attached to a scene mechanism with its joint values per target.  fp64 kin_ik_coll_batch(_scene) vs the CPU
restatement (oracle or_ik_coll_batch, the sphere rows in the kernel's order): equal iteration counts, angles
within 1e-7, |dp| / |rot| / min distance within 1e-9, generic and plan-specialised kernels.  The reference's
own scene (PR2, both arms, 14 joints + base) needs the network-downloaded PR2 model; these scenes have the
same structure (two arms off one torso, a base, an articulated fridge).  Sphere placement is
parity-unpinned (no meshes)."""
import numpy as np
import pytest
import torch

from conftest import ARM, golden

import kinhip

pytestmark = pytest.mark.gpu

KW = dict(margin=0.02, band=0.01, weight=1.0, feas=1e-6, max_iters=96, lam=1e-2, tol_pos=1e-4, tol_rot=1e-4,
          max_step=0.5, with_rot=2, restarts=2, seed=7)

# two arms of four revolute joints off a prismatic torso (the PR2 / fridge_demo.jl structure, smaller)
TWO_ARM = """<robot name="twoarm">
  <link name="base_link"/><link name="torso"/>
  <link name="l1"/><link name="l2"/><link name="l3"/><link name="l4"/><link name="l_grip"/>
  <link name="r1"/><link name="r2"/><link name="r3"/><link name="r4"/><link name="r_grip"/>
  <joint name="torso_joint" type="prismatic"><parent link="base_link"/><child link="torso"/>
    <origin xyz="0 0 0.8"/><axis xyz="0 0 1"/><limit lower="0" upper="0.3" effort="1" velocity="1"/></joint>
  <joint name="l_j1" type="revolute"><parent link="torso"/><child link="l1"/><origin xyz="0.05 0.2 0.2"/>
    <axis xyz="0 0 1"/><limit lower="-2" upper="2" effort="1" velocity="1"/></joint>
  <joint name="l_j2" type="revolute"><parent link="l1"/><child link="l2"/><origin xyz="0.1 0 0"/>
    <axis xyz="0 1 0"/><limit lower="-1.5" upper="1.5" effort="1" velocity="1"/></joint>
  <joint name="l_j3" type="continuous"><parent link="l2"/><child link="l3"/><origin xyz="0.3 0 0"/>
    <axis xyz="1 0 0"/></joint>
  <joint name="l_j4" type="revolute"><parent link="l3"/><child link="l4"/><origin xyz="0.05 0 0"/>
    <axis xyz="0 1 0"/><limit lower="-2.2" upper="2.2" effort="1" velocity="1"/></joint>
  <joint name="l_tool" type="fixed"><parent link="l4"/><child link="l_grip"/><origin xyz="0.3 0 0"/></joint>
  <joint name="r_j1" type="revolute"><parent link="torso"/><child link="r1"/><origin xyz="0.05 -0.2 0.2"/>
    <axis xyz="0 0 1"/><limit lower="-2" upper="2" effort="1" velocity="1"/></joint>
  <joint name="r_j2" type="revolute"><parent link="r1"/><child link="r2"/><origin xyz="0.1 0 0"/>
    <axis xyz="0 1 0"/><limit lower="-1.5" upper="1.5" effort="1" velocity="1"/></joint>
  <joint name="r_j3" type="continuous"><parent link="r2"/><child link="r3"/><origin xyz="0.3 0 0"/>
    <axis xyz="1 0 0"/></joint>
  <joint name="r_j4" type="revolute"><parent link="r3"/><child link="r4"/><origin xyz="0.05 0 0"/>
    <axis xyz="0 1 0"/><limit lower="-2.2" upper="2.2" effort="1" velocity="1"/></joint>
  <joint name="r_tool" type="fixed"><parent link="r4"/><child link="r_grip"/><origin xyz="0.3 0 0"/></joint>
</robot>
"""
TWO_ARM_Q = ["r_j1", "r_j2", "r_j3", "r_j4", "torso_joint", "l_j1", "l_j2", "l_j3", "l_j4"]
TWO_ARM_SPHERES = [(side + n, c, r) for side in ("l", "r") for n, c, r in
                   (("2", (0.1, 0, 0), 0.05), ("2", (0.22, 0, 0), 0.05), ("4", (0.1, 0, 0), 0.045),
                    ("4", (0.25, 0, 0), 0.04))]


def _pose(t, yaw=0.0):
    T = np.eye(4)
    c, s = np.cos(yaw), np.sin(yaw)
    T[:3, :3] = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
    T[:3, 3] = t
    return T


def _col(T):
    return np.concatenate([T[:3, :3].T.reshape(-1), T[:3, 3]])


class Scene:
    """The robot on the GPU side and the oracle's restatement, the same spheres on both."""

    def __init__(self, urdf_path, q_names, spheres, with_base=False):
        import oracle as O
        self.O = O
        self.m = kinhip.parse_urdf(urdf_path, with_base=with_base)
        self.q = [self.m.find_joint(n) for n in q_names]
        self.sscc = kinhip.SweptSphereCollisionChecker(self.m)
        self.tree = O.parse_urdf_tree(urdf_path)
        self.om = O.OracleMech(self.tree, with_base=with_base)
        self.sph, self.rad, self.par = [], [], []
        for name, c, r in spheres:
            self.sscc.add_coll_sphere(self.m.find_link(name), c, r)
            T = np.eye(4)
            T[:3, 3] = c
            self.sph.append(self.om.add_new_link(self.tree.link_id(name), T))
            self.rad.append(r)
            self.par.append(self.tree.link_id(name))
        self.ids = [self.tree.joint_id(n) for n in q_names]
        self.nd = len(q_names) + (3 if with_base else 0)

    def sphere_centres(self, q, link_names):
        """World centres of the spheres at configuration q (oracle FK)."""
        self.om.set_joint_angles(self.ids, q)
        return [self.om.get_transform(s)[:3, 3] for s in self.sph]

    def check(self, link, tg, Q1, sdf, box=None, boxes=None, spec=False, lanes=0, scene_q=None, kw=KW,
              min_conv=0.5, knife_edge=0.01, q_alt=None):
        """GPU vs oracle.  Equal iteration counts on all but `knife_edge` of the targets: a sphere the penalty
        holds at the band's edge (d -> margin + band, where its row switches on and off) sits on a
        switching surface, and last-bit differences between the kernel's FMA sums and the oracle's can
        flip its row on a step -- the two runs then part.  On the targets with equal counts: converged
        answers' angles within 1e-7 and err rows within 1e-9; unconverged ones return the lowest-merit
        attempt, and attempts that end in the same constrained minimum tie in merit to the last bits, so
        there the merits (from the err rows) agree to 1e-9 while the angles may be another tying attempt's."""
        plan = kinhip.CollisionIKPlan(self.sscc, self.m.find_link(link), self.q, dtype=torch.float64)
        if spec:
            plan.specialize()
        dev = Q1.device
        tgt = torch.tensor(tg, dtype=torch.float64, device=dev).contiguous()
        Q, it, err = plan.ik_coll(sdf, tgt, torch.empty_like(Q1), Q0=Q1, lanes=lanes, scene_q=scene_q, Q_alt=q_alt,
                                  **kw)
        rq, rit, rerr = self.O.ik_coll_batch(self.om, box, Q1.cpu().numpy(), self.ids, self.tree.link_id(link), tg,
                                             self.sph, self.rad, sdfs=boxes, sphere_parents=self.par,
                                             q_alt=None if q_alt is None else q_alt.cpu().numpy(), **kw)
        it = it.cpu().numpy()
        q, e = Q.cpu().numpy(), err.cpu().numpy()
        conv = it <= kw["max_iters"]
        assert conv.mean() >= min_conv, conv.mean()
        same = it == rit
        assert (~same).mean() <= knife_edge, (np.where(~same)[0], it[~same], rit[~same])
        c = same & conv
        np.testing.assert_allclose(q[:, c], rq[:, c], atol=1e-7)
        np.testing.assert_allclose(e[:, c], rerr[:, c], atol=1e-9)
        u = same & ~conv
        w2 = kw["weight"] ** 2

        def merit(x):
            return x[0] ** 2 + x[1] ** 2 + w2 * np.maximum(kw["margin"] - x[2], 0.0) ** 2
        np.testing.assert_allclose(merit(e[:, u]), merit(rerr[:, u]), rtol=1e-9, atol=1e-12)
        return Q, it, err


def _fridge_box():
    import oracle as O
    fr = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
    sdf = kinhip.fridge_sdf(fr)
    return sdf, O.OracleUnionSDF([b.pose for b in sdf.sdfs], [b.width for b in sdf.sdfs])


def _fridge_targets(rng, N):
    tg = np.zeros((12, N))
    for k in range(N):
        tg[:, k] = _col(_pose((rng.uniform(0.9, 1.05), rng.uniform(-0.12, 0.12), rng.uniform(1.15, 1.32)),
                              rng.uniform(-0.3, 0.3)))
    return tg


def _stage1(sc, link, tg, dev):
    """Stage-1 solutions (collision-free DLS on the same plan) as the stage-2 seeds."""
    plan = kinhip.CollisionIKPlan(sc.sscc, sc.m.find_link(link), sc.q, dtype=torch.float64)
    tgt = torch.tensor(tg, dtype=torch.float64, device=dev).contiguous()
    Q1 = torch.zeros((sc.nd, tg.shape[1]), dtype=torch.float64, device=dev)
    plan.ik_dls(tgt, Q1, max_iters=64, restarts=3, seed=2, with_rot=2)  # (in place: other columns stay 0)
    return Q1


@pytest.mark.parametrize("spec,lanes", [(False, 0), (True, 0), (True, 1), (True, 64)])
def test_fetch_arm_with_head_spheres(spec, lanes):
    """Spheres on two moving chains of Fetch: the arm (torso .. wrist) and the head (head_pan, head_tilt are
    q columns too: they move no target, only head spheres -- the solver moves them out of a box placed on
    the head of the stage-1 solution).  The tree branches at torso_lift_link (a saved branch frame)."""
    import oracle as O
    names = ARM + ["head_pan_joint", "head_tilt_joint"]
    spheres = kinhip.FETCH_ARM_SPHERES + [("head_pan_link", (0.1, 0.0, 0.1), 0.1),
                                          ("head_tilt_link", (0.05, 0.0, 0.0), 0.09),
                                          ("head_tilt_link", (0.15, 0.0, 0.0), 0.06)]
    sc = Scene(golden("fetch.urdf"), names, spheres)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(41)
    N = 256
    tg = _fridge_targets(rng, N)
    Q1 = _stage1(sc, "gripper_link", tg, dev)
    # a box on the head of target 0's stage-1 solution: every target's head starts in collision
    c = sc.sphere_centres(Q1[:, 0].cpu().numpy(), None)[-2]
    sdf0, _ = _fridge_box()
    sdf = kinhip.UnionSDF(sdf0.sdfs + [kinhip.BoxSDF(_pose(c + [0.0, 0.0, 0.05]), (0.12, 0.3, 0.12))])
    box = O.OracleUnionSDF([b.pose for b in sdf.sdfs], [b.width for b in sdf.sdfs])
    Q, it, err = sc.check("gripper_link", tg, Q1, sdf, box=box, spec=spec, lanes=lanes)
    # the head joints moved (they only move head spheres)
    moved = np.abs(Q.cpu().numpy()[8:10] - Q1.cpu().numpy()[8:10]).max(axis=0)
    assert (moved[it <= KW["max_iters"]] > 1e-3).mean() > 0.5


@pytest.mark.parametrize("with_base", [False, True])
@pytest.mark.parametrize("spec,lanes", [(False, 0), (True, 0), (True, 16)])
def test_two_arm_tree(tmp_path, spec, lanes, with_base):
    """Two arms off one torso (fridge_demo.jl's joints = vcat(rarm, larm) with spheres on both arms): the
    target is the left gripper, the right arm's joints move only right-arm spheres.  A box sits on the
    right forearm of the stage-1 solutions, so the solve must move the right arm while the left holds its
    pose.  With a planar base: 9 joints + 3 base columns = 12 variables."""
    import oracle as O
    path = tmp_path / "twoarm.urdf"
    path.write_text(TWO_ARM)
    sc = Scene(str(path), TWO_ARM_Q, TWO_ARM_SPHERES, with_base=with_base)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(43)
    N = 300
    # reachable left-gripper poses (FK of random torso / left-arm angles, and base offsets): four arm joints
    # and the torso cannot reach an arbitrary 6-D pose without the base
    qt = np.zeros((sc.nd, N))
    qt[4] = rng.uniform(0.05, 0.25, N)
    qt[5:9] = np.stack([rng.uniform(-0.8, 0.8, N), rng.uniform(-0.6, 0.6, N), rng.uniform(-1.0, 1.0, N),
                        rng.uniform(-1.2, 1.2, N)])
    if with_base:
        qt[9:12] = np.stack([rng.uniform(-0.2, 0.2, N), rng.uniform(-0.2, 0.2, N), rng.uniform(-0.3, 0.3, N)])
    tg = sc.om.fk_batch(qt, sc.ids, [sc.tree.link_id("l_grip")])[0]
    Q1 = _stage1(sc, "l_grip", tg, dev)
    Q1[:4] = torch.tensor([0.3, 0.4, 0.0, 0.6], dtype=torch.float64, device=dev)[:, None]  # right arm start
    # a box around r4's first sphere of target 0's start (off its centre: at the centre every face is
    # nearest and the SDF gradient is a tie that last-bit differences break either way)
    c = sc.sphere_centres(Q1[:, 0].cpu().numpy(), None)[6] + np.array([0.02, -0.015, 0.01])
    sdf = kinhip.UnionSDF([kinhip.BoxSDF(_pose(c), (0.1, 0.1, 0.1)),
                           kinhip.BoxSDF(_pose((0.6, 0.0, 0.4)), (0.8, 1.2, 0.05))])
    box = O.OracleUnionSDF([b.pose for b in sdf.sdfs], [b.width for b in sdf.sdfs])
    d0, _ = O.coll_batch(sc.om, box, Q1.cpu().numpy(), sc.ids, sc.sph[4:], sc.rad[4:], with_grad=False)
    hit = d0.min(axis=0) < KW["margin"]  # the targets whose right arm starts too close to the box
    assert hit.sum() >= 5, hit.sum()
    Q, it, err = sc.check("l_grip", tg, Q1, sdf, box=box, spec=spec, lanes=lanes)
    conv = it <= KW["max_iters"]
    moved = np.abs(Q.cpu().numpy()[:4] - Q1.cpu().numpy()[:4]).max(axis=0)
    assert (moved[conv & hit] > 1e-3).mean() > 0.5  # the right arm left the box


@pytest.mark.parametrize("alt", [False, True])
@pytest.mark.parametrize("spec", [False, True])
def test_fetch_with_base_in_fridge(spec, alt):
    """Fetch with its planar base (8 joints + x, y, theta): stage 2 in the fridge scene of
    test/test_inverse_kinematics.jl:52-86, the base a variable of every sphere row.  alt: a second start
    pose per target (kin_ik_coll_batch_alt; random angles within the limits and base offsets) that restart
    attempt 1 starts from, joints and base, on the GPU and in the oracle."""
    sc = Scene(golden("fetch.urdf"), ARM, kinhip.FETCH_ARM_SPHERES, with_base=True)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(47)
    N = 256
    tg = _fridge_targets(rng, N)
    Q1 = _stage1(sc, "gripper_link", tg, dev)
    sdf, box = _fridge_box()
    q_alt = None
    if alt:
        lo = np.array([j.lower_limit for j in sc.q])
        hi = np.array([j.upper_limit for j in sc.q])
        lo, hi = np.where(np.isfinite(lo), lo, -np.pi), np.where(np.isfinite(hi), hi, np.pi)
        qa = np.concatenate([rng.uniform(lo[:, None], hi[:, None], (len(lo), N)),
                             rng.uniform(-0.1, 0.1, (3, N))])
        q_alt = torch.tensor(qa, dtype=torch.float64, device=dev).contiguous()
    sc.check("gripper_link", tg, Q1, sdf, box=box, spec=spec, q_alt=q_alt)


def test_door_angle_per_target():
    """fridge_demo.jl's scene with the door angle a per-target input (kin_ik_coll_batch_scene: the fridge
    as a UnionSDF attached to its mechanism, scene columns door + base per target) vs the oracle's static
    union of each target's fridge state (oracle.fridge_boxes)."""
    import oracle as O
    sc = Scene(golden("fetch.urdf"), ARM, kinhip.FETCH_ARM_SPHERES)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(53)
    N = 192
    tg = _fridge_targets(rng, N)
    Q1 = _stage1(sc, "gripper_link", tg, dev)
    fr = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
    asdf = kinhip.AttachedUnionSDF(fr, [fr.find_joint("door_joint")])
    doors = rng.uniform(1.5, 2.4, N)
    scene_q = torch.tensor(np.stack([doors, np.full(N, 1.2), np.zeros(N), np.zeros(N)]), dtype=torch.float64,
                           device=dev).contiguous()
    ft = O.parse_urdf_tree(golden("fridge.urdf"))
    boxes = [O.OracleUnionSDF(*O.fridge_boxes(ft, door_angle=d, base=(1.2, 0.0, 0.0))) for d in doors]
    sc.check("gripper_link", tg, Q1, asdf, box=None, boxes=boxes, scene_q=scene_q)
    # one scene state for the whole batch == the static union of that state
    plan = kinhip.CollisionIKPlan(sc.sscc, sc.m.find_link("gripper_link"), sc.q, dtype=torch.float64)
    tgt = torch.tensor(tg, dtype=torch.float64, device=dev).contiguous()
    a = plan.ik_coll(asdf, tgt, torch.empty_like(Q1), Q0=Q1, scene_q=scene_q[:, 0].contiguous(), **KW)
    fr2 = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
    b = plan.ik_coll(kinhip.fridge_sdf(fr2, door_angle=float(doors[0])), tgt, torch.empty_like(Q1), Q0=Q1, **KW)
    # (the attached union places its boxes by FK on the device, the static one on the host: last-bit
    # differences, so the iteration counts may split on a handful of targets)
    ia, ib = a[1].cpu().numpy(), b[1].cpu().numpy()
    same = ia == ib
    assert same.mean() > 0.98
    np.testing.assert_allclose(a[0].cpu().numpy()[:, same], b[0].cpu().numpy()[:, same], atol=1e-7)


@pytest.mark.parametrize("spec", [False, True])
def test_unsolvable_targets_return_the_best_attempt(spec):
    """a target no attempt can solve (inside a box: the pose and the constraint conflict)
    returns the attempt whose end state has the lowest merit |dp|^2 + |rot|^2 + w^2 max(0, margin - d)^2,
    as NLopt returns its best point -- not the last re-drawn attempt.  Same rule in the oracle; the
    returned err rows are the returned state's."""
    import oracle as O
    sc = Scene(golden("fetch.urdf"), ARM, kinhip.FETCH_ARM_SPHERES)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(59)
    N = 128
    tg = _fridge_targets(rng, N)
    Q1 = _stage1(sc, "gripper_link", tg, dev)
    sdf0, _ = _fridge_box()
    # a box around the target region: the gripper's spheres cannot reach the targets without entering it
    sdf = kinhip.UnionSDF(sdf0.sdfs + [kinhip.BoxSDF(_pose((0.98, 0.0, 1.235)), (0.4, 0.4, 0.25))])
    box = O.OracleUnionSDF([b.pose for b in sdf.sdfs], [b.width for b in sdf.sdfs])
    Q, it, err = sc.check("gripper_link", tg, Q1, sdf, box=box, spec=spec, min_conv=0.0)
    fail = it > KW["max_iters"]
    assert fail.mean() > 0.5
    # err of a failed target is the returned state's: recompute with the oracle
    q = Q.cpu().numpy()
    gl = sc.tree.link_id("gripper_link")
    pose = sc.om.fk_batch(q, sc.ids, [gl])[0]
    dp = np.linalg.norm(pose[9:] - tg[9:], axis=0)
    np.testing.assert_allclose(dp[fail], err.cpu().numpy()[0][fail], atol=1e-9)
    d, _ = O.coll_batch(sc.om, box, q, sc.ids, sc.sph, sc.rad, with_grad=False)
    np.testing.assert_allclose(d.min(0)[fail], err.cpu().numpy()[2][fail], atol=1e-9)


def test_padded_ldq_beyond_the_narrow_bound():
    """the collision-aware IK with a leading dimension whose row offsets pass 2^31 bytes (fp64,
    8 columns, ld = 2^25 + 64) -- every load and store of the kernel is 64-bit safe; the answers equal
    those of a dense call."""
    sc = Scene(golden("fetch.urdf"), ARM, kinhip.FETCH_ARM_SPHERES)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(61)
    N = 256
    tg = _fridge_targets(rng, N)
    Q1 = _stage1(sc, "gripper_link", tg, dev)
    sdf, _ = _fridge_box()
    plan = kinhip.CollisionIKPlan(sc.sscc, sc.m.find_link("gripper_link"), sc.q, dtype=torch.float64).specialize()
    tgt = torch.tensor(tg, dtype=torch.float64, device=dev).contiguous()
    ref = plan.ik_coll(sdf, tgt, torch.empty_like(Q1), Q0=Q1, **KW)
    ld = (1 << 25) + 64
    big0 = torch.zeros((8, ld), dtype=torch.float64, device=dev)
    big = torch.zeros((8, ld), dtype=torch.float64, device=dev)
    big0[:, :N] = Q1
    got = plan.ik_coll(sdf, tgt, big[:, :N], Q0=big0[:, :N], **KW)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]) and torch.equal(got[2], ref[2])
    del big, big0


# ---- the reference's own PR2 shape: both arms (14 joints) + the planar base = 17 variables ----

def _pr2_scene(with_base=True):
    """tests/golden/pr2_two_arms.urdf at reset_manip_pose (src/models.jl:59-70): the torso (not a batch
    column) at 0.3; q columns = rarm_joints then larm_joints (test_inverse_kinematics.jl:33, 60)."""
    names = kinhip.PR2_RARM_JOINTS + kinhip.PR2_LARM_JOINTS
    sc = Scene(golden("pr2_two_arms.urdf"), names, kinhip.PR2_ARM_SPHERES, with_base=with_base)
    torso = sc.m.find_joint("torso_lift_joint")
    base = [0.0, 0.0, 0.0] if with_base else []
    sc.m.set_joint_angles([torso], [0.3] + base)
    sc.om.set_joint_angles([sc.tree.joint_id("torso_lift_joint")], [0.3] + base)
    r, l, _ = kinhip.PR2_MANIP_POSE
    q0 = np.deg2rad(np.array(r + l))
    if with_base:
        q0 = np.concatenate([q0, np.zeros(3)])
    return sc, q0


def _pr2_fridge_targets(rng, N):
    """test_inverse_kinematics.jl:67-68: Transform((0, 0, 1.2)) * pose_fridge (fridge base at (1.2, 0, 0)),
    perturbed per target."""
    tg = np.zeros((12, N))
    for k in range(N):
        tg[:, k] = _col(_pose((1.2 + rng.uniform(-0.06, 0.0), rng.uniform(-0.06, 0.06), 1.2 + rng.uniform(-0.05, 0.05)),
                              rng.uniform(-0.2, 0.2)))
    return tg


def test_pr2_plan_accepts_seventeen_variables():
    """kin_coll_ik_plan_create takes the reference's call shape: 14 arm joints + base = 17 variables (the
    cap was 12), every sphere of both arms' collision links; the fp32 and fp64 plans specialise."""
    sc, _ = _pr2_scene()
    for dt in (torch.float32, torch.float64):
        plan = kinhip.CollisionIKPlan(sc.sscc, sc.m.find_link("l_gripper_tool_frame"), sc.q, dtype=dt)
        assert plan.n_qcols == 17
        plan.specialize()
        assert plan.specialized & kinhip.KIN_SPEC_IK_COLL_SCENE


@pytest.mark.parametrize("spec,lanes", [(False, 0), (True, 0), (True, 1), (True, 64)])
def test_pr2_two_arms_with_base_door_per_target(spec, lanes):
    """The reference's collision-aware IK call (test/test_inverse_kinematics.jl:52-86, fridge_demo.jl:13-37):
    PR2 with its base, joints = vcat(rarm, larm), spheres on both arms' collision links, the l_gripper_tool_frame
    target inside the fridge -- and the fridge door angle per target (kin_ik_coll_batch_scene, the fridge as a
    UnionSDF attached to its mechanism).  fp64 vs the oracle's or_ik_coll_batch over the static union of each
    target's fridge state: equal iteration counts, angles 1e-7."""
    import oracle as O
    sc, q0 = _pr2_scene()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(67)
    N = 128
    tg = _pr2_fridge_targets(rng, N)
    link = "l_gripper_tool_frame"
    plan = kinhip.CollisionIKPlan(sc.sscc, sc.m.find_link(link), sc.q, dtype=torch.float64)
    tgt = torch.tensor(tg, dtype=torch.float64, device=dev).contiguous()
    Q0 = torch.tensor(np.repeat(q0[:, None], N, 1), dtype=torch.float64, device=dev).contiguous()
    Q1 = torch.empty_like(Q0)
    plan.ik_dls(tgt, Q1, Q0=Q0, max_iters=64, restarts=3, seed=2, with_rot=2)  # stage 1 (rarm columns pass through)
    Q1[:7] = Q0[:7]
    fr = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
    asdf = kinhip.AttachedUnionSDF(fr, [fr.find_joint("door_joint")])
    doors = rng.uniform(1.6, 2.4, N)
    scene_q = torch.tensor(np.stack([doors, np.full(N, 1.2), np.zeros(N), np.zeros(N)]), dtype=torch.float64,
                           device=dev).contiguous()
    ft = O.parse_urdf_tree(golden("fridge.urdf"))
    boxes = [O.OracleUnionSDF(*O.fridge_boxes(ft, door_angle=d, base=(1.2, 0.0, 0.0))) for d in doors]
    Q, it, err = sc.check(link, tg, Q1, asdf, box=None, boxes=boxes, spec=spec, lanes=lanes, scene_q=scene_q)
    conv = it <= KW["max_iters"]
    # the reference's acceptance on the converged targets: |dp| < 1e-3 and every sphere clear (vals > -1e-5)
    e = err.cpu().numpy()
    assert (e[0][conv] < 1e-3).all() and (e[2][conv] > KW["margin"] - 1e-5).all()
    # the bistage form (CollisionIKPlan.solve): restart attempt 1 from the pose stage 1 started from
    # (kin_ik_coll_batch_alt, q_alt = Q0) -- iterates vs the oracle again, and it converges at least as often
    Qa, ita, erra = sc.check(link, tg, Q1, asdf, box=None, boxes=boxes, spec=spec, lanes=lanes, scene_q=scene_q,
                             q_alt=Q0)
    conva = ita <= KW["max_iters"]
    print(f"PR2 door per target: converged {conv.mean():.3f}, with attempt 1 from the start pose {conva.mean():.3f}")
    assert conva.mean() >= conv.mean()
    a0 = torch.tensor(it <= KW["max_iters"] // (KW["restarts"] + 1), device=dev)  # solved by attempt 0: unchanged
    assert torch.equal(Qa[:, a0], Q[:, a0]) and torch.equal(erra[:, a0], err[:, a0])
    assert (ita[a0.cpu().numpy()] == it[a0.cpu().numpy()]).all()


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_scene_specialized_equals_generic(dtype):
    """kin_ik_coll_batch_scene's specialised S x G-lane kernels (KIN_SPEC_IK_COLL_SCENE) against the generic
    kernel: bit-identical angles, iteration counts and errors for every lane layout (the fridge door per
    target, Fetch's arm)."""
    sc = Scene(golden("fetch.urdf"), ARM, kinhip.FETCH_ARM_SPHERES)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(71)
    N = 700
    tg = _fridge_targets(rng, N)
    Q1 = _stage1(sc, "gripper_link", tg, dev).to(dtype)
    fr = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
    asdf = kinhip.AttachedUnionSDF(fr, [fr.find_joint("door_joint")])
    scene_q = torch.tensor(np.stack([rng.uniform(1.5, 2.4, N), np.full(N, 1.2), np.zeros(N), np.zeros(N)]),
                           dtype=dtype, device=dev).contiguous()
    tgt = torch.tensor(tg, dtype=dtype, device=dev).contiguous()
    gen = kinhip.CollisionIKPlan(sc.sscc, sc.m.find_link("gripper_link"), sc.q, dtype=dtype)
    spc = kinhip.CollisionIKPlan(sc.sscc, sc.m.find_link("gripper_link"), sc.q, dtype=dtype).specialize()
    kw = dict(KW, restarts=3)
    ref = gen.ik_coll(asdf, tgt, torch.empty_like(Q1), Q0=Q1, scene_q=scene_q, lanes=1, **kw)
    it = ref[1].cpu().numpy()
    assert (it <= kw["max_iters"]).mean() > 0.5
    for lanes in (0, 1, 4, 16, 64):
        got = spc.ik_coll(asdf, tgt, torch.empty_like(Q1), Q0=Q1, scene_q=scene_q, lanes=lanes, **kw)
        for a, b in zip(got, ref):
            assert torch.equal(a, b), lanes
    # with a second start pose (kin_ik_coll_batch_alt) for attempt 1: every layout still bit-identical
    Qa = torch.zeros_like(Q1)
    ref = gen.ik_coll(asdf, tgt, torch.empty_like(Q1), Q0=Q1, scene_q=scene_q, lanes=1, Q_alt=Qa, **kw)
    for lanes in (0, 1, 4, 16, 64):
        got = spc.ik_coll(asdf, tgt, torch.empty_like(Q1), Q0=Q1, scene_q=scene_q, lanes=lanes, Q_alt=Qa, **kw)
        for a, b in zip(got, ref):
            assert torch.equal(a, b), ("alt", lanes)


@pytest.mark.parametrize("with_base", [False, True])
@pytest.mark.parametrize("with_rot", [0, 2])
def test_pr2_dls_no_collision_vs_oracle(with_base, with_rot):
    """The reference's "no collision" PR2 case (test/test_inverse_kinematics.jl:29-49): kin_ik_dls_batch over
    joints = vcat(rarm, larm) (the right arm's 7 columns cannot move l_gripper_tool_frame: left untouched) with
    and without the base, from reset_manip_pose towards (0.6, 0.7, 0.8) (perturbed per target), position only and
    the reference's rpy objective.  fp64 iterates vs the oracle's or_ik_dls_batch (equal iteration counts, angles
    1e-7) and the reference's acceptance |dp| < 1e-3 on the converged targets."""
    sc, q0 = _pr2_scene(with_base)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(73)
    N = 256
    tg = np.zeros((12, N))
    for k in range(N):
        tg[:, k] = _col(_pose((0.6 + rng.uniform(-0.05, 0.05), 0.7 + rng.uniform(-0.05, 0.05),
                               0.8 + rng.uniform(-0.05, 0.05)), rng.uniform(-0.2, 0.2)))
    link = sc.m.find_link("l_gripper_tool_frame")
    plan = sc.m.plan(sc.q, out_links=[link], jac_link=link, dtype=torch.float64)
    tgt = torch.tensor(tg, dtype=torch.float64, device=dev).contiguous()
    Q = torch.tensor(np.repeat(q0[:, None], N, 1), dtype=torch.float64, device=dev).contiguous()
    kw = dict(max_iters=64, restarts=3, seed=9, lam=1e-2, tol_pos=1e-4, tol_rot=1e-4, max_step=0.5)
    Q, it, err = plan.ik_dls(tgt, Q, with_rot=with_rot, **kw)
    rq, rit, rerr = sc.om.ik_dls_batch(np.repeat(q0[:, None], N, 1), sc.ids, sc.tree.link_id("l_gripper_tool_frame"),
                                       tg, with_rot=with_rot, **kw)
    it = it.cpu().numpy()
    np.testing.assert_array_equal(it, rit)
    np.testing.assert_allclose(Q.cpu().numpy(), rq, atol=1e-7)
    conv = it <= kw["max_iters"]
    assert conv.mean() > 0.9, conv.mean()
    assert (err.cpu().numpy()[0][conv] < 1e-3).all()
    np.testing.assert_array_equal(Q.cpu().numpy()[:7], np.repeat(q0[:7, None], N, 1))  # the right arm untouched
