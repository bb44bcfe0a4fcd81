"""Replay of the Julia shim's plan caching (kinematics.jl_amd/julia/KinematicsHIP.jl: HIPModel, sync!,
baked_angles, cached_plan!, plan!) over the same C-ABI calls through ctypes, in the order a Julia caller
makes them: the HIPModel is created once, a batched call stages and caches a plan, the caller moves a
joint the batch does not drive (set_joint_angles(m, [head_pan], ...), src/mechanism.jl:223-231) and
calls again, then grows the tree with add_new_link (src/mechanism.jl:238-267) and calls again.  The
reference reads m.angles and the tree on every call (src/algorithm.jl:1-37), so every answer must match
the oracle at the mechanism's state of that moment (1e-12, fp64).  A replay without sync! (the round-2
shim) is run beside it to show the sequence does catch a stale plan.

The shim's single-target calls -- the reference's own signatures inverse_kinematics!(hm, link, joints,
target::Transform; ftol, with_rot) -> (q, status), its collision form (sscc, sdf; use_bistage) and
compute_coll_dists -- are replayed the same way for all three testsets of test/test_inverse_kinematics.jl,
asserting the reference's checks verbatim (VERDICT r05 "next" 2).

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
    """The Julia Mechanism's state the shim reads: links / joints (kinhip's Python mirror as data),
    m.angles and m.base_pose.  Its own C model is not used by the replay."""

    def __init__(self, path, with_base=False):
        self.m = kinhip.parse_urdf(path, with_base=with_base)
        self.with_base = with_base
        self.angles = np.zeros(len(self.m.joints))
        self.base_pose = np.zeros(3)

    def get_joint_angles(self, ids):
        """get_joint_angles(m, joints) (src/mechanism.jl:203-221): the joints' angles, then the base pose."""
        return np.array([self.angles[i - 1] for i in ids] + (list(self.base_pose) if self.with_base else []))

    def set_joint_angles(self, ids, q):
        """set_joint_angles(m, joints, angles) (src/mechanism.jl:223-231)."""
        q = np.asarray(q, np.float64)
        for i, a in zip(ids, q[:len(ids)]):
            self.angles[i - 1] = a
        if self.with_base:
            self.base_pose = q[len(ids):len(ids) + 3].copy()

    def add_new_link(self, name, parent, T):
        self.m.add_new_link(kinhip.Link(name), parent, T)
        self.angles = np.append(self.angles, 0.0)  # push!(m.angles, 0.0)


def model_handle(mech):
    """KinematicsHIP.jl model_handle: kin_model_create + kin_model_set_angles(m.angles)."""
    arrs = mech.m._tree_arrays()
    d = K.TreeDesc(len(mech.m.links), len(mech.m.joints), *[_p(a).value for a in arrs], int(mech.with_base))
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

    def coll_plan(self, sph_ids, radii, qj):
        """KinematicsHIP.jl coll_plan!: kin_coll_plan_create(KinCollDesc(Float64, ids, spheres, radii)) + specialise."""
        qj, sph = np.ascontiguousarray(qj, np.int32), np.ascontiguousarray(sph_ids, np.int32)
        r = np.ascontiguousarray(radii, np.float64)
        key = ("coll", qj.tobytes(), sph.tobytes())

        def make():
            h = C.c_void_p()
            d = K.CollDesc(K.KIN_F64, qj.size, _p(qj).value, sph.size, _p(sph).value, None, _p(r).value)
            K.check(K.lib().kin_coll_plan_create(self.handle, C.byref(d), C.byref(h)))
            K.lib().kin_plan_specialize(h, 0)
            return h

        return self.cached_plan(make, key, qj)

    def collik_plan(self, sph_ids, radii, link_id, qj):
        """KinematicsHIP.jl collik_plan!: kin_coll_ik_plan_create (NULL sphere arrays when there are none)."""
        qj, sph = np.ascontiguousarray(qj, np.int32), np.ascontiguousarray(sph_ids, np.int32)
        r = np.ascontiguousarray(radii, np.float64)
        key = ("collik", qj.tobytes(), sph.tobytes(), link_id)

        def make():
            h = C.c_void_p()
            d = K.CollDesc(K.KIN_F64, qj.size, _p(qj).value, sph.size, _p(sph).value if sph.size else None, None,
                           _p(r).value if r.size else None)
            K.check(K.lib().kin_coll_ik_plan_create(self.handle, C.byref(d), link_id, C.byref(h)))
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
    kin_ik_coll_batch_alt (restart attempt 1 from Q0) with one door angle per target (scene columns door, base x, y, theta) -- replayed
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
        K.check(K.lib().kin_ik_coll_batch_alt(p, sdf, C.byref(prm), C.byref(cp), targets.data_ptr(), N,
                                              scene_q.data_ptr(), N, Q1.data_ptr(), Q0.data_ptr(), Q.data_ptr(), N,
                                              N, iters.data_ptr(), err.data_ptr(), N, None))
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
                                    margin=0.02, band=0.0, weight=1.0, feas=1e-6, sdfs=boxes, sphere_parents=opar,
                                    q_alt=np.zeros((8, N)), **kw)
    it = iters.cpu().numpy()
    same = it == rit
    assert (~same).mean() <= 0.01, (np.where(~same)[0], it[~same], rit[~same])
    c = same & (it <= 64)
    assert c.mean() > 0.8
    np.testing.assert_allclose(Q.cpu().numpy()[:, c], rq[:, c], atol=1e-7)
    np.testing.assert_allclose(err.cpu().numpy()[:, c], rerr[:, c], atol=1e-9)


# ---- the reference's single-target calls (KinematicsHIP.jl "the reference's own single-target calls") ----

def _dev():
    return torch.device("cuda", 0)


def target_batch(T):
    """KinematicsHIP.jl target_batch: the 3x4 column-major 12-vector, a batch of one."""
    T = np.asarray(T, np.float64)
    return torch.tensor([T[r, c] for c in range(4) for r in range(3)], dtype=torch.float64, device=_dev()).reshape(12, 1)


def angles_batch(mech, ids):
    """KinematicsHIP.jl angles_batch: get_joint_angles(m, joints) as a batch of one."""
    return torch.tensor(mech.get_joint_angles(ids), dtype=torch.float64, device=_dev()).reshape(-1, 1).contiguous()


def ik_ftol(hm, link_id, ids, T, ftol=1e-5, with_rot=True, max_iters=200, lam=1e-2, max_step=0.5):
    """KinematicsHIP.jl inverse_kinematics!(hm, link, joints, target_pose::Transform; ftol, with_rot), line for
    line: the trace launch, NLopt's ftol_abs rule on every iterate's objective, the launch of k steps."""
    mech = hm.mech
    p = hm.plan(ids, [link_id], link_id, ids, K.KIN_WITH_ROT)
    tgt = target_batch(T)
    q0 = angles_batch(mech, ids)
    q = torch.empty_like(q0)
    iters = torch.empty(1, dtype=torch.int32, device=_dev())
    M = int(max_iters)
    mode = 2 if with_rot else 0
    trace = torch.full((2 * (M + 1), 1), float("nan"), dtype=torch.float64, device=_dev())
    prm = K.IkParams(M, lam, 0.0, 0.0, max_step, mode, 0, 0, 1, 0, 0.0)
    K.check(K.lib().kin_ik_dls_batch_trace(p, C.byref(prm), tgt.data_ptr(), 1, q0.data_ptr(), q.data_ptr(), 1, 1,
                                           iters.data_ptr(), trace.data_ptr(), 1, None))
    tr = trace[:, 0].cpu().numpy()
    f = tr[0::2] ** 2 + tr[1::2] ** 2
    status, k = ":MAXEVAL_REACHED", M
    for kk in range(1, M + 1):
        if abs(f[kk - 1] - f[kk]) < ftol:
            status, k = ":FTOL_REACHED", kk
            break
    prm_k = K.IkParams(k, lam, 0.0, 0.0, max_step, mode, 0, 0, 1, 0, 0.0)
    K.check(K.lib().kin_ik_dls_batch_from(p, C.byref(prm_k), tgt.data_ptr(), 1, q0.data_ptr(), q.data_ptr(), 1, 1,
                                          iters.data_ptr(), None, 1, None))
    qv = q[:, 0].cpu().numpy()
    mech.set_joint_angles(ids, qv)
    return qv, status


def ik_coll(hm, link_id, ids, T, sscc, sdf_h, use_bistage=True, ftol=1e-5, with_rot=True, max_iters=200, lam=1e-2,
            max_step=0.5, margin=0.02):
    """KinematicsHIP.jl inverse_kinematics!(hm, link, joints, target_pose::Transform, sscc, sdf; use_bistage, ftol,
    with_rot) for a static sdf (HIPSDF(UnionSDF) = kin_sdf_create_boxes), line for line.  `sscc` =
    (sphere link ids, radii)."""
    mech = hm.mech
    q_start = angles_batch(mech, ids)
    if use_bistage:
        ik_ftol(hm, link_id, ids, T, ftol=ftol, with_rot=with_rot, max_iters=max_iters, lam=lam, max_step=max_step)
    sph, rad = sscc
    p = hm.collik_plan(sph, rad, link_id, ids)
    tgt = target_batch(T)
    q0 = angles_batch(mech, ids)
    q = torch.empty_like(q0)
    iters = torch.empty(1, dtype=torch.int32, device=_dev())
    err = torch.empty((3, 1), dtype=torch.float64, device=_dev())
    prm = K.IkParams(max_iters, lam, 1e-6, 1e-6, max_step, 2 if with_rot else 0, 3, 0, 0, 0, 0.0)
    cprm = K.IkCollParams(margin, 0.0, 1.0, 1e-6)
    K.check(K.lib().kin_ik_coll_batch_alt(p, sdf_h, C.byref(prm), C.byref(cprm), tgt.data_ptr(), 1, None, 0,
                                          q0.data_ptr(), q_start.data_ptr() if use_bistage else None, q.data_ptr(),
                                          1, 1, iters.data_ptr(), err.data_ptr(), 1, None))
    qv = q[:, 0].cpu().numpy()
    mech.set_joint_angles(ids, qv)
    return qv, (":FTOL_REACHED" if int(iters[0]) <= max_iters else ":MAXEVAL_REACHED")


def compute_coll_dists(hm, sscc, ids, sdf_h):
    """KinematicsHIP.jl compute_coll_dists(hm, sscc, joints, sdf): coll_plan! + kin_coll_batch on a batch of one at
    the mechanism's current angles; no spheres -> an empty vector."""
    sph, rad = sscc
    if len(sph) == 0:
        return np.zeros(0)
    p = hm.coll_plan(sph, rad, ids)
    Q = angles_batch(hm.mech, ids)
    vals = torch.empty((len(sph), 1), dtype=torch.float64, device=_dev())
    K.check(K.lib().kin_coll_batch(p, sdf_h, float("inf"), Q.data_ptr(), 1, 1, vals.data_ptr(), 1, None, 1, None,
                                   None))
    return vals[:, 0].cpu().numpy()


def _isapprox(x, y, atol):
    """Julia's isapprox(x, y; atol) on vectors (rtol = 0 when atol > 0): norm(x - y) <= atol."""
    return float(np.linalg.norm(np.asarray(x) - np.asarray(y))) <= atol


def _pose2angles(T):
    """test_inverse_kinematics.jl:44: RotZYX(rotation(pose)) -> [theta1, theta2, theta3] (yaw, pitch, roll)."""
    return O.rpy(T)[::-1]


def _oracle_pose(path, mech, ids, link_name):
    """get_transform(mech, link) -- the reference's CPU path (the oracle) at the mechanism's state."""
    tree = O.parse_urdf_tree(path)
    om = O.OracleMech(tree, with_base=mech.with_base)
    nz = [j.id for j in mech.m.joints[:len(tree.joint_names)] if mech.angles[j.id - 1] != 0.0]
    if nz or mech.with_base:
        om.set_joint_angles(nz, [mech.angles[i - 1] for i in nz] + (list(mech.base_pose) if mech.with_base else []))
    return om.get_transform(tree.link_id(link_name))


def _translation(T):
    return np.asarray(T)[:3, 3]


def _transform(t):
    T = np.eye(4)
    T[:3, 3] = t
    return T


def _reset_manip_pose(robot):
    """reset_manip_pose (src/models.jl:59-70)."""
    r, l, torso = kinhip.PR2_MANIP_POSE
    ids = [robot.m.find_joint(n).id for n in kinhip.PR2_RARM_JOINTS + kinhip.PR2_LARM_JOINTS + ["torso_lift_joint"]]
    av = list(np.deg2rad(r)) + list(np.deg2rad(l)) + [torso] + ([0.0, 0.0, 0.0] if robot.with_base else [])
    robot.set_joint_angles(ids, av)


@pytest.mark.parametrize("with_base", [False, True])
def test_replay_reference_ik_fetch(with_base):
    """test/test_inverse_kinematics.jl:1-25, through the shim's inverse_kinematics!(hm, link, joints, target)."""
    path = golden("fetch.urdf")
    mech = Mech(path, with_base=with_base)
    hm = HIPModel(mech)
    try:
        joints = [mech.m.find_joint(n).id for n in ARM]
        link = mech.m.find_link("gripper_link").id
        target_pose = _transform((0.3, -0.4, 1.2))
        q_goal, status = ik_ftol(hm, link, joints, target_pose, with_rot=True)
        assert status == ":FTOL_REACHED"
        mech.set_joint_angles(joints, q_goal)
        pose_now = _oracle_pose(path, mech, joints, "gripper_link")
        assert _isapprox(O.rpy(pose_now), O.rpy(target_pose), atol=1e-3)
        assert _isapprox(_translation(pose_now), _translation(target_pose), atol=1e-3)
    finally:
        hm.close()


@pytest.mark.parametrize("with_base", [False, True])
def test_replay_reference_ik_pr2_no_collision(with_base):
    """test/test_inverse_kinematics.jl:29-50 (tests/golden/pr2_two_arms.urdf for load_pr2: network-only),
    both with_rot calls in sequence on the same robot, ftol = 1e-7."""
    path = golden("pr2_two_arms.urdf")
    robot = Mech(path, with_base=with_base)
    hm = HIPModel(robot)
    try:
        link = robot.m.find_link("l_gripper_tool_frame").id
        joints = [robot.m.find_joint(n).id for n in kinhip.PR2_RARM_JOINTS + kinhip.PR2_LARM_JOINTS]
        _reset_manip_pose(robot)
        pose_target = _transform((0.6, 0.7, 0.8))
        for with_rot in (False, True):
            _, status = ik_ftol(hm, link, joints, pose_target, with_rot=with_rot, ftol=1e-7)
            assert status == ":FTOL_REACHED", with_rot
            pose_actual = _oracle_pose(path, robot, joints, "l_gripper_tool_frame")
            pos_diff = _translation(pose_target) - _translation(pose_actual)
            assert np.linalg.norm(pos_diff) < 1e-3, (with_rot, pos_diff)
            if with_rot and with_base:
                rot_diff = _pose2angles(pose_target) - _pose2angles(pose_actual)
                assert np.linalg.norm(rot_diff) < 1e-3, rot_diff
    finally:
        hm.close()


def _fridge_scene():
    """test_inverse_kinematics.jl:53-70: the fridge with its base, door 2.0 at base (1.2, 0, 0); the target
    Transform((0, 0, 1.2)) * pose_fridge; sdf = UnionSDF(fridge) at that state (HIPSDF(sdf) snapshot)."""
    fridge = kinhip.parse_urdf(golden("fridge.urdf"), with_base=True)
    sdf = kinhip.fridge_sdf(fridge, door_angle=2.0, base=(1.2, 0.0, 0.0))  # kin_sdf_create_boxes of the boxes
    ft = O.parse_urdf_tree(golden("fridge.urdf"))
    of = O.OracleMech(ft, with_base=True)
    of.set_joint_angles([ft.joint_id("door_joint")], [2.0, 1.2, 0.0, 0.0])
    pose_fridge = of.get_transform(ft.link_id("base_link"))
    pose_target = _transform((0.0, 0.0, 1.2)) @ pose_fridge
    boxes = O.OracleUnionSDF(*O.fridge_boxes(ft, door_angle=2.0, base=(1.2, 0.0, 0.0)))
    return sdf, pose_target, boxes


@pytest.mark.parametrize("spheres", ["verbatim", "arm_spheres"])
def test_replay_reference_ik_pr2_with_collision(spheres):
    """test/test_inverse_kinematics.jl:52-86 through the shim's collision form and compute_coll_dists.
    "verbatim": the reference's checker exactly as its test builds it -- `(add_coll_links(sscc, link) for link
    in collision_links)` (:63) is an un-iterated generator, so no sphere is added and the constraint is
    empty; "arm_spheres": the spheres that line means to add (kinhip.PR2_ARM_SPHERES on both arms' collision
    links, build-defined: the reference fits them to meshes), so stage 2 enforces them.  The reference's own
    checks: :FTOL_REACHED, norm(pos_diff) < 1e-3, norm(rot_diff) < 1e-3, all(compute_coll_dists .> -1e-5); the
    distances also equal the oracle's at the answer."""
    path = golden("pr2_two_arms.urdf")
    sdf, pose_target, boxes = _fridge_scene()
    robot = Mech(path, with_base=True)
    sph, rad, par, centres = [], [], [], []
    if spheres == "arm_spheres":
        for name, c, r in kinhip.PR2_ARM_SPHERES:
            robot.add_new_link(f"sphere_{len(sph)}", robot.m.find_link(name), _transform(c))
            sph.append(robot.m.find_link(f"sphere_{len(sph)}").id)
            rad.append(r)
            par.append(name)
            centres.append(c)
    hm = HIPModel(robot)
    try:
        joints = [robot.m.find_joint(n).id for n in kinhip.PR2_RARM_JOINTS + kinhip.PR2_LARM_JOINTS]
        _reset_manip_pose(robot)
        link = robot.m.find_link("l_gripper_tool_frame").id
        q_goal, status = ik_coll(hm, link, joints, pose_target, (sph, rad), sdf._h, with_rot=True, use_bistage=True)
        assert status == ":FTOL_REACHED"
        pose_actual = _oracle_pose(path, robot, joints, "l_gripper_tool_frame")
        pos_diff = _translation(pose_target) - _translation(pose_actual)
        assert np.linalg.norm(pos_diff) < 1e-3, pos_diff
        rot_diff = _pose2angles(pose_target) - _pose2angles(pose_actual)
        assert np.linalg.norm(rot_diff) < 1e-3, rot_diff
        vals = compute_coll_dists(hm, (sph, rad), joints, sdf._h)
        assert np.all(vals > -1e-5), vals
        assert vals.size == len(sph)
        if sph:  # the same distances from the CPU restatement at the answer
            tree = O.parse_urdf_tree(path)
            om = O.OracleMech(tree, with_base=True)
            osph = []
            for name, c in zip(par, centres):
                osph.append(om.add_new_link(tree.link_id(name), _transform(c)))
            oids = [tree.joint_id(n) for n in kinhip.PR2_RARM_JOINTS + kinhip.PR2_LARM_JOINTS]
            om.set_joint_angles([tree.joint_id("torso_lift_joint")], [kinhip.PR2_MANIP_POSE[2], 0.0, 0.0, 0.0])
            q = robot.get_joint_angles(joints).reshape(-1, 1)
            od = O.coll_batch(om, boxes, q, oids, osph, rad)[0][:, 0]
            np.testing.assert_allclose(vals, od, atol=1e-9)
            print(f"arm spheres: min distance {vals.min():.4f} (margin 0.02)")
    finally:
        hm.close()


@pytest.mark.parametrize("spheres", ["verbatim", "arm_spheres"])
def test_python_mirror_reference_pr2_with_collision(spheres):
    """The same reference testset through the Python mirror (kinhip.inverse_kinematics_ with kinhip.UnionSDF,
    kinhip.compute_coll_dists), the reference's checks verbatim."""
    sdf, pose_target, _ = _fridge_scene()
    robot = kinhip.parse_urdf(golden("pr2_two_arms.urdf"), with_base=True)
    joints = [robot.find_joint(n) for n in kinhip.PR2_RARM_JOINTS + kinhip.PR2_LARM_JOINTS]
    sscc = kinhip.SweptSphereCollisionChecker(robot)
    if spheres == "arm_spheres":
        for name, c, r in kinhip.PR2_ARM_SPHERES:
            sscc.add_coll_sphere(robot.find_link(name), c, r)
    r, l, torso = kinhip.PR2_MANIP_POSE
    robot.set_joint_angles(joints + [robot.find_joint("torso_lift_joint")],
                           list(np.deg2rad(r)) + list(np.deg2rad(l)) + [torso, 0.0, 0.0, 0.0])
    link = robot.find_link("l_gripper_tool_frame")
    q_goal, status = kinhip.inverse_kinematics_(robot, link, joints, pose_target, sscc, sdf, with_rot=True,
                                                use_bistage=True)
    assert status == ":FTOL_REACHED"
    pose_actual = kinhip.get_transform(robot, link)
    assert np.linalg.norm(_translation(pose_target) - _translation(pose_actual)) < 1e-3
    assert np.linalg.norm(_pose2angles(pose_target) - _pose2angles(pose_actual)) < 1e-3
    vals = kinhip.compute_coll_dists(sscc, joints, sdf)
    assert np.all(vals > -1e-5), vals


# ---- the reference's plan_trajectory through GPUSDF (KinematicsHIP.jl "plan_trajectory with the collision
# queries on the GPU") ----

def gpusdf_ineq_const(hm, sscc, ids, sdf_h, margin, n_dof, n_wp, xi, val_vec, jac_mat):
    """KinematicsHIP.jl (this::IneqConst)(xi::Vector, val_vec::Vector, jac_mat::Matrix) for a GPUSDF, line for
    line: X = reshape(xi, n_dof, n_wp); Xi = permutedims(X) on the device ((n_wp, n_dof) column-major: row d of a
    C-contiguous (n_dof, n_wp) array); coll_plan! + kin_ineq_const_batch; the block-diagonal fill; the
    mechanism left at the last waypoint."""
    sph, rad = sscc
    n_coll = len(sph)
    if n_coll == 0:
        return
    X = np.asarray(xi, np.float64).reshape(n_wp, n_dof).T  # Julia reshape(xi, (n_dof, n_wp))
    Xi = torch.tensor(np.ascontiguousarray(X), dtype=torch.float64, device=_dev())
    vals = torch.empty((n_coll, n_wp), dtype=torch.float64, device=_dev())         # Julia (n_wp, n_coll)
    jac = torch.empty((n_coll, n_dof, n_wp), dtype=torch.float64, device=_dev())   # Julia (n_wp, n_dof, n_coll)
    p = hm.coll_plan(sph, rad, ids)
    K.check(K.lib().kin_ineq_const_batch(p, sdf_h, float(margin), Xi.data_ptr(), n_wp, n_wp, vals.data_ptr(), n_wp,
                                         jac.data_ptr(), n_wp, None))
    v, J = vals.cpu().numpy(), jac.cpu().numpy()
    for i in range(n_wp):
        val_vec[n_coll * i:n_coll * (i + 1)] = v[:, i]
        jac_mat[n_dof * i:n_dof * (i + 1), n_coll * i:n_coll * (i + 1)] = J[:, :, i].T  # Julia J[i, :, :]
    hm.mech.set_joint_angles(ids, X[:, -1])


PLANNING_COLL_LINKS = ["wrist_flex_link", "torso_lift_link", "upperarm_roll_link", "elbow_flex_link"]


@pytest.mark.parametrize("with_base", [False, True])
def test_replay_reference_planning_through_gpusdf(with_base):
    """test/test_planning.jl's planning_test(with_base, :SCIPY) with `boxsdf` wrapped as GPUSDF(boxsdf): the
    reference's plan_trajectory (src/planning.jl:332-401) unchanged -- its compute_coll_dists asserts on the
    start and goal (the GPUSDF method: the shim's compute_coll_dists(hm, ...)), construct_problem, the :SCIPY
    minimize(f, xi_init, SLSQP, [ineq g, eq h], ftol) with g = scipynize(IneqConst), whose call is the shim's
    batched GPUSDF method (replayed above).  Asserted: the replayed IneqConst equals the Python mirror's bit
    for bit and the oracle's restatement (values 1e-9), at the straight line and at the answer; SLSQP succeeds;
    the answer keeps its end points and every waypoint satisfies the reference's :NLOPT check
    (compute_coll_dists .> -1e-2).  The spheres are build-defined (FETCH_LINK_SPHERES) and so the goal is the
    first collision-free batched IK answer for the reference's target (as tests/test_planning.py)."""
    from scipy.optimize import minimize

    path = golden("fetch.urdf")
    mech = Mech(path, with_base=with_base)
    sph, rad, osph = [], [], []
    tree = O.parse_urdf_tree(path)
    om = O.OracleMech(tree, with_base=with_base)
    for n in PLANNING_COLL_LINKS:  # add_coll_links(sscc, find_link(mech, n)) (src/collision.jl:39-49)
        for c, r in kinhip.FETCH_LINK_SPHERES[n]:
            name = f"{n}_sphere_{len(sph)}"
            mech.add_new_link(name, mech.m.find_link(n), _transform(c))
            sph.append(mech.m.find_link(name).id)
            rad.append(r)
            osph.append(om.add_new_link(tree.link_id(n), _transform(c)))
    sscc = (sph, rad)
    joints = [mech.m.find_joint(n).id for n in ARM]
    n_dof = len(joints) + (3 if with_base else 0)
    boxsdf = kinhip.UnionSDF([kinhip.BoxSDF(_transform((0.4, -0.25, 0.7)), (0.05, 0.05, 0.5))])  # HIPSDF(boxsdf)
    obox = O.OracleUnionSDF([_transform((0.4, -0.25, 0.7))], [[0.05, 0.05, 0.5]])
    # the mirror's IneqConst on its own mechanism with the same spheres
    mm = kinhip.parse_urdf(path, with_base=with_base)
    msscc = kinhip.SweptSphereCollisionChecker(mm)
    for n in PLANNING_COLL_LINKS:
        kinhip.add_coll_links(msscc, mm.find_link(n))
    mjoints = [mm.find_joint(n) for n in ARM]
    n_wp, margin = 10, 2e-2
    hm = HIPModel(mech)
    try:
        q_start = mech.get_joint_angles(joints)
        # goal: the first collision-free answer of a batched IK for (0.3, -0.4, 1.2) without rotation
        gl = mm.find_link("gripper_link")
        plan = mm.plan(mjoints, out_links=[gl], jac_link=gl, jac_joints=mjoints, dtype=torch.float64)
        N = 256
        g = torch.Generator().manual_seed(11)
        Q0 = (torch.rand((n_dof, N), generator=g, dtype=torch.float64) * 2 - 1).to(_dev())
        if with_base:
            Q0[8:] = 0.0
        tgt = torch.tensor(np.repeat(_transform((0.3, -0.4, 1.2))[:3, :4].T.reshape(12, 1), N, axis=1), device=_dev())
        Q, it, _ = plan.ik_dls(tgt, Q0.contiguous(), with_rot=False, max_iters=64)
        _, _, mn = msscc.plan(mjoints, dtype=torch.float64).run(boxsdf, Q, dists=False, min_dist=True)
        ok = ((it <= 64) & (mn > 0.05)).nonzero()
        assert ok.numel() > 0
        q_goal = Q[:, int(ok[0, 0])].cpu().numpy()
        # plan_trajectory(sscc, joints, GPUSDF(boxsdf), q_start, q_goal, n_wp; ftol_abs=1e-5, solver=:SCIPY)
        for q in (q_start, q_goal):
            mech.set_joint_angles(joints, q)
            assert np.all(compute_coll_dists(hm, sscc, joints, boxsdf._h) > 0.0)
        xi_init = kinhip.create_straight_trajectory(q_start, q_goal, n_wp)
        F = kinhip.Objective(n_wp, np.ones(n_dof))
        H = kinhip.EqConst(n_wp, [kinhip.ConfigurationConstraint(1, n_dof, q_start),
                                  kinhip.ConfigurationConstraint(n_wp, n_dof, q_goal)])
        g_val = np.zeros(n_wp * len(sph))
        g_jac = np.zeros((n_dof * n_wp, n_wp * len(sph)))
        G = kinhip.IneqConst(msscc, mjoints, boxsdf, n_wp, margin)

        def check_g(xi):
            gpusdf_ineq_const(hm, sscc, joints, boxsdf._h, margin, n_dof, n_wp, xi, g_val, g_jac)
            G(xi, G.val_vec, G.jac_mat)
            assert np.array_equal(g_val, G.val_vec) and np.array_equal(g_jac, G.jac_mat)
            rv, _ = O.ineq_const(om, obox, xi, [tree.joint_id(n) for n in ARM], osph, rad, n_wp, margin)
            np.testing.assert_allclose(g_val, rv, atol=1e-9)
            np.testing.assert_array_equal(mech.get_joint_angles(joints), np.asarray(xi).reshape(n_wp, n_dof)[-1])

        check_g(xi_init)
        grad = np.zeros(xi_init.size)

        def g_fun(xi):
            gpusdf_ineq_const(hm, sscc, joints, boxsdf._h, margin, n_dof, n_wp, xi, g_val, g_jac)
            return g_val.copy()

        def h_fun(xi):
            H(xi, H.val_vec, H.jac_mat)
            return H.val_vec.copy()

        cons = [{"type": "ineq", "fun": g_fun, "jac": lambda xi: (g_fun(xi), g_jac.T.copy())[1]},
                {"type": "eq", "fun": h_fun, "jac": lambda xi: (h_fun(xi), H.jac_mat.T.copy())[1]}]
        res = minimize(lambda x: F(x, grad), xi_init, method="SLSQP", constraints=cons, options={"ftol": 1e-5})
        assert res.success, res.message
        q_seq = res.x.reshape(n_wp, n_dof).T
        np.testing.assert_allclose(q_seq[:, 0], q_start, atol=1e-6)
        np.testing.assert_allclose(q_seq[:, -1], q_goal, atol=1e-6)
        check_g(res.x)
        for i in range(n_wp):  # the reference's :NLOPT checks (test_planning.jl:39-44)
            mech.set_joint_angles(joints, q_seq[:, i])
            assert np.all(compute_coll_dists(hm, sscc, joints, boxsdf._h) > -1e-2), i
    finally:
        hm.close()
