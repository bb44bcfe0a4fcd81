"""Replay of the Julia shim's plan caching (kinematics.jl_amd/julia/KinematicsHIP.jl: HIPModel, sync!,
baked_angles, cached_plan!, plan!) over the same C-ABI calls through ctypes, in the order a Julia caller
makes them: the HIPModel is created once, a batched call stages and caches a plan, the caller moves a
joint the batch does not drive (set_joint_angles(m, [head_pan], ...), src/mechanism.jl:223-231) and
calls again, then grows the tree with add_new_link (src/mechanism.jl:238-267) and calls again.  The
reference reads m.angles and the tree on every call (src/algorithm.jl:1-37), so every answer must match
the oracle at the mechanism's state of that moment (1e-12, fp64).  A replay without sync! (the round-2
shim) is run beside it to show the sequence does catch a stale plan.

Julia is not in this image; tests/test_julia_shim.py checks statically that every batched call of the
shim obtains its plan through cached_plan! (and so through sync!)."""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle as O
from conftest import ARM, golden

import kinhip
from kinhip import _lib as K

pytestmark = pytest.mark.gpu


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class Mech:
    """The Julia Mechanism's state the shim reads: links / joints (kinhip's Python mirror as data) and
    m.angles.  Its own C model is not used by the replay."""

    def __init__(self, path):
        self.m = kinhip.parse_urdf(path)
        self.angles = np.zeros(len(self.m.joints))

    def add_new_link(self, name, parent, T):
        self.m.add_new_link(kinhip.Link(name), parent, T)
        self.angles = np.append(self.angles, 0.0)  # push!(m.angles, 0.0)


def model_handle(mech):
    """KinematicsHIP.jl model_handle: kin_model_create + kin_model_set_angles(m.angles)."""
    arrs = mech.m._tree_arrays()
    d = K.TreeDesc(len(mech.m.links), len(mech.m.joints), *[_p(a).value for a in arrs], 0)
    h = C.c_void_p()
    K.check(K.lib().kin_model_create(C.byref(d), C.byref(h)))
    a = np.ascontiguousarray(mech.angles, np.float64)
    K.check(K.lib().kin_model_set_angles(h, _p(a)))
    return h


class HIPModel:
    """KinematicsHIP.jl HIPModel with sync! / baked_angles / cached_plan! / plan! (line for line);
    `follow=False` is the round-2 shim: model and plans never follow the Mechanism."""

    def __init__(self, mech, follow=True):
        self.mech, self.follow = mech, follow
        self.handle = model_handle(mech)
        self.plans = {}
        self.angles = mech.angles.copy()
        self.n_links = len(mech.m.links)

    def free_plans(self):
        for p, _ in self.plans.values():
            K.lib().kin_plan_destroy(p)
        self.plans.clear()

    def close(self):
        self.free_plans()
        K.lib().kin_model_destroy(self.handle)

    def sync(self):
        m = self.mech
        if len(m.m.links) != self.n_links or len(m.angles) != len(self.angles):
            self.free_plans()
            K.lib().kin_model_destroy(self.handle)
            self.handle = model_handle(m)
            self.n_links = len(m.m.links)
            self.angles = m.angles.copy()
        elif not np.array_equal(m.angles, self.angles):
            a = np.ascontiguousarray(m.angles, np.float64)
            K.check(K.lib().kin_model_set_angles(self.handle, _p(a)))
            self.angles = m.angles.copy()

    def baked_angles(self, qj):
        a = self.mech.angles.copy()
        a[np.asarray(qj) - 1] = 0.0
        return a

    def cached_plan(self, make, key, qj):
        if self.follow:
            self.sync()
        baked = self.baked_angles(qj)
        hit = self.plans.get(key)
        if hit is not None:
            if not self.follow or np.array_equal(hit[1], baked):
                return hit[0]
            K.lib().kin_plan_destroy(hit[0])
            del self.plans[key]
        p = make()
        self.plans[key] = (p, baked)
        return p

    def plan(self, qj, outs, jl, jj, flags):
        qj, outs, jj = (np.ascontiguousarray(x, np.int32) for x in (qj, outs, jj))
        key = (qj.tobytes(), outs.tobytes(), jl, jj.tobytes(), flags)

        def make():
            h = C.c_void_p()
            d = K.PlanDesc(K.KIN_F64, qj.size, _p(qj).value, outs.size, _p(outs).value, jl, jj.size, _p(jj).value,
                           flags)
            K.check(K.lib().kin_plan_create(self.handle, C.byref(d), C.byref(h)))
            K.lib().kin_plan_specialize(h, 0)
            return h

        return self.cached_plan(make, key, qj)

    def get_transform(self, link_ids, joint_ids, Q):
        """Kinematics.get_transform(hm, links, joints, Q): poses (n_links, 12, N)."""
        N = Q.shape[1]
        poses = torch.empty((len(link_ids), 12, N), dtype=torch.float64, device=Q.device)
        p = self.plan(joint_ids, link_ids, 0, [], 0)
        K.check(K.lib().kin_plan_run(p, Q.data_ptr(), Q.stride(0), N, poses.data_ptr(), N, None, 0, None))
        return poses

    def get_jacobian(self, link_id, joint_ids, Q):
        """Kinematics.get_jacobian!(hm, link, joints, true, J, Q; pose): (pose, J) with J zero-filled."""
        N = Q.shape[1]
        J = torch.zeros((len(joint_ids), 6, N), dtype=torch.float64, device=Q.device)
        pose = torch.empty((1, 12, N), dtype=torch.float64, device=Q.device)
        p = self.plan(joint_ids, [link_id], link_id, joint_ids, K.KIN_WITH_ROT)
        K.check(K.lib().kin_plan_run(p, Q.data_ptr(), Q.stride(0), N, pose.data_ptr(), N, J.data_ptr(), N, None))
        return pose, J


def _oracle(mech, tree, extra):
    om = O.OracleMech(tree)
    nz = [j.id for j in mech.m.joints[:len(tree.joint_names)] if mech.angles[j.id - 1] != 0.0]
    if nz:
        om.set_joint_angles(nz, [mech.angles[i - 1] for i in nz])
    for parent, T in extra:
        om.add_new_link(parent, T)
    return om


@pytest.mark.parametrize("follow", [True, False])
def test_shim_sequence_follows_the_mechanism(follow):
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dev = torch.device("cuda", 0)
    tree = O.parse_urdf_tree(golden("fetch.urdf"))
    mech = Mech(golden("fetch.urdf"))
    m = mech.m
    arm = [m.find_joint(n).id for n in ARM]
    gl, head = m.find_link("gripper_link").id, m.find_link("head_tilt_link").id
    hp, ht = m.find_joint("head_pan_joint").id, m.find_joint("head_tilt_joint").id
    N = 512
    g = torch.Generator().manual_seed(11)
    Q = (torch.rand((8, N), generator=g, dtype=torch.float64) * 2 - 1).to(dev)
    Qn = Q.cpu().numpy()
    hm = HIPModel(mech, follow=follow)
    extra = []
    stale = []

    def check():
        torch.cuda.synchronize()
        om = _oracle(mech, tree, extra)
        links = [gl, head] + [lid for _, _, lid in extra_ids]
        try:
            P = hm.get_transform(links, arm, Q).cpu().numpy()
        except kinhip.KinError:
            if follow:
                raise
            stale.append(True)  # the stale C model does not know the new link (KIN_E_KEY)
            return None
        ref = om.fk_batch(Qn, arm, links)
        pose, J = hm.get_jacobian(gl, arm, Q)
        ps, js = om.fk_jac_batch(Qn, arm, gl, arm, True, False)
        errs = [np.abs(P - ref).max(), np.abs(pose.cpu().numpy() - ps).max(), np.abs(J.cpu().numpy() - js).max()]
        stale.append(max(errs) > 1e-12)
        if follow:
            assert max(errs) <= 1e-12, errs
        return P

    extra_ids = []
    try:
        p0 = check()  # plans staged and cached
        p0b = check()  # the same cached plans
        assert np.array_equal(p0, p0b)
        assert len(hm.plans) == 2
        mech.angles[hp - 1] = 0.6  # set_joint_angles(m, [head_pan, head_tilt], ...): not batch columns
        mech.angles[ht - 1] = -0.25
        check()
        T = np.eye(4)
        T[:3, 3] = [0.04, 0.01, -0.03]
        mech.add_new_link("tool_tip", m.find_link("gripper_link"), T)  # add_new_link
        extra.append((gl, T))
        extra_ids.append((gl, T, m.find_link("tool_tip").id))
        check()
        mech.angles[hp - 1] = -0.4  # and once more after the tree grew
        check()
    finally:
        hm.close()
    # without sync! the cached plans keep the old head angles (the round-2 shim's bug) -- and the
    # tree query after add_new_link fails on the stale C model
    if not follow:
        assert any(stale)


def test_shim_collision_ik_with_attached_fridge():
    """KinematicsHIP.jl's inverse_kinematics!(hm, link, joints, targets, Q0, sscc, sdf::HIPSDF; scene_q) with
    the reference's UnionSDF(fridge) (test/test_inverse_kinematics.jl:52-86, fridge_demo.jl:13-37): the shim's
    exact C-ABI sequence -- HIPSDF(fridge, [door_joint]) = kin_model_create + kin_sdf_create_attached;
    the cached plan = kin_coll_ik_plan_create + kin_plan_specialize(0); stage 1 kin_ik_dls_batch_from; stage 2
    kin_ik_coll_batch_scene with one door angle per target (scene columns door, base x, y, theta) -- replayed
    through ctypes with the shim's default keywords, against the oracle: stage 1 or_ik_dls_batch, stage 2
    or_ik_coll_batch over each target's static fridge union (fp64, equal iteration counts, angles 1e-7)."""
    import oracle as O
    from kinhip import collision as KC

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dev = torch.device("cuda", 0)
    # the robot (Fetch, arm spheres) and the scene: HIPModel(robot), HIPSDF(fridge, [door_joint])
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    sscc = kinhip.SweptSphereCollisionChecker(m)
    kinhip.add_fetch_arm_spheres(sscc)
    arm = [m.find_joint(n) for n in ARM]
    gl = m.find_link("gripper_link")
    m._sync_angles()
    fr = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
    fr._sync_angles()
    links = [l for l in fr.links if l.geometric_meta_data is not None and hasattr(l.geometric_meta_data, "extents")]
    jids = np.array([fr.find_joint("door_joint").id], np.int32)
    lids = np.array([l.id for l in links], np.int32)
    org = np.ascontiguousarray(np.array([np.asarray(l.geometric_meta_data.origin, np.float64).T.reshape(16)
                                         for l in links]).reshape(-1))
    wid = np.ascontiguousarray(np.array([l.geometric_meta_data.extents for l in links], np.float64).reshape(-1))
    sdf = C.c_void_p()
    K.check(K.lib().kin_sdf_create_attached(fr._model, 1, _p(jids), lids.size, _p(lids), _p(org), _p(wid),
                                            C.byref(sdf)))
    # cached_plan!: kin_coll_ik_plan_create(KinCollDesc(Float64, ids, sphere links, radii)) + specialise (0)
    ids = np.array([j.id for j in arm], np.int32)
    sph = np.array([l.id for l in sscc.sphere_links], np.int32)
    rad = np.asarray(sscc.sphere_radii, np.float64)
    d = K.CollDesc(K.KIN_F64, ids.size, _p(ids).value, sph.size, _p(sph).value, None, _p(rad).value)
    p = C.c_void_p()
    K.check(K.lib().kin_coll_ik_plan_create(m._model, C.byref(d), gl.id, C.byref(p)))
    K.check(K.lib().kin_plan_specialize(p, 0))
    N = 160
    rng = np.random.default_rng(79)
    tg = np.zeros((12, N))
    for k in range(N):
        T = np.eye(4)
        c, s = np.cos(rng.uniform(-0.3, 0.3)), np.sin(rng.uniform(-0.3, 0.3))
        T[:3, :3] = [[c, -s, 0], [s, c, 0], [0, 0, 1]]
        T[:3, 3] = (rng.uniform(0.9, 1.05), rng.uniform(-0.12, 0.12), rng.uniform(1.15, 1.32))
        tg[:, k] = np.concatenate([T[:3, :3].T.reshape(-1), T[:3, 3]])
    doors = rng.uniform(1.5, 2.4, N)
    targets = torch.tensor(tg, dtype=torch.float64, device=dev).contiguous()
    scene_q = torch.tensor(np.stack([doors, np.full(N, 1.2), np.zeros(N), np.zeros(N)]), dtype=torch.float64,
                           device=dev).contiguous()
    Q0 = torch.zeros((8, N), dtype=torch.float64, device=dev)
    Q1, Q = torch.empty_like(Q0), torch.empty_like(Q0)
    iters = torch.empty(N, dtype=torch.int32, device=dev)
    err = torch.empty((3, N), dtype=torch.float64, device=dev)
    # the shim's defaults: max_iters=64, lambda=1e-2, tol 1e-3, max_step=0.5, rpy_objective -> with_rot 2,
    # restarts=3, seed=0, lanes=0, damp_err=0; margin=0.02, band=0, weight=1, feas=1e-6
    prm = K.IkParams(64, 1e-2, 1e-3, 1e-3, 0.5, 2, 3, 0, 0, 0)
    cp = K.IkCollParams(0.02, 0.0, 1.0, 1e-6)
    try:
        K.check(K.lib().kin_ik_dls_batch_from(p, C.byref(prm), targets.data_ptr(), N, Q0.data_ptr(), Q1.data_ptr(),
                                              N, N, iters.data_ptr(), err.data_ptr(), N, None))
        K.check(K.lib().kin_ik_coll_batch_scene(p, sdf, C.byref(prm), C.byref(cp), targets.data_ptr(), N,
                                                scene_q.data_ptr(), N, Q1.data_ptr(), Q.data_ptr(), N, N,
                                                iters.data_ptr(), err.data_ptr(), N, None))
        torch.cuda.synchronize()
    finally:
        K.lib().kin_plan_destroy(p)
        K.lib().kin_sdf_destroy(sdf)
    tree = O.parse_urdf_tree(golden("fetch.urdf"))
    om = O.OracleMech(tree)
    osph, opar = [], []
    for name, c, _ in KC.FETCH_ARM_SPHERES:
        T = np.eye(4)
        T[:3, 3] = c
        osph.append(om.add_new_link(tree.link_id(name), T))
        opar.append(tree.link_id(name))
    oids = [tree.joint_id(n) for n in ARM]
    kw = dict(max_iters=64, lam=1e-2, tol_pos=1e-3, tol_rot=1e-3, max_step=0.5, with_rot=2, restarts=3, seed=0)
    q1, _, _ = om.ik_dls_batch(np.zeros((8, N)), oids, tree.link_id("gripper_link"), tg, **kw)
    np.testing.assert_allclose(Q1.cpu().numpy(), q1, atol=1e-7)
    ft = O.parse_urdf_tree(golden("fridge.urdf"))
    boxes = [O.OracleUnionSDF(*O.fridge_boxes(ft, door_angle=dd, base=(1.2, 0.0, 0.0))) for dd in doors]
    rq, rit, rerr = O.ik_coll_batch(om, None, q1, oids, tree.link_id("gripper_link"), tg, osph, list(rad),
                                    margin=0.02, band=0.0, weight=1.0, feas=1e-6, sdfs=boxes, sphere_parents=opar, **kw)
    it = iters.cpu().numpy()
    same = it == rit
    assert (~same).mean() <= 0.01, (np.where(~same)[0], it[~same], rit[~same])
    c = same & (it <= 64)
    assert c.mean() > 0.8
    np.testing.assert_allclose(Q.cpu().numpy()[:, c], rq[:, c], atol=1e-7)
    np.testing.assert_allclose(err.cpu().numpy()[:, c], rerr[:, c], atol=1e-9)
