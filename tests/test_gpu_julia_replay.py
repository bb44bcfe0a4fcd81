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
