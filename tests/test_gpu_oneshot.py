"""The one-shot C-ABI entry points kin_get_transform_batch / kin_get_jacobian_batch (include/kinhip.h; the
drop-in for get_transform / get_jacobian! over a batch, src/algorithm.jl:1-4, 83-114) vs the oracle,
including their per-model plan cache: reuse, and invalidation by kin_model_set_angles (angles of joints
the batch does not drive) and kin_model_add_link.  Also the Python mirror's argument checks that keep a
host / other-device pointer from reaching a kernel."""
import ctypes as C

import numpy as np
import pytest
import torch

import oracle as O
from conftest import ARM, golden

import kinhip
from kinhip import _lib as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda", 0)


def _oracle_with(tree, angles_by_id, extra_links=()):
    om = O.OracleMech(tree)
    ids = list(angles_by_id)
    if ids:
        om.set_joint_angles(ids, [angles_by_id[i] for i in ids])
    for parent, T in extra_links:
        om.add_new_link(parent, T)
    return om


def test_oneshot_transform_and_jacobian_cache_and_invalidation(dev):
    tree = O.parse_urdf_tree(golden("fetch.urdf"))
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    gl, head = m.find_link("gripper_link"), m.find_link("head_tilt_link")
    links = [gl, head, m.find_link("r_gripper_finger_link")]
    N = 1000
    g = torch.Generator().manual_seed(3)
    Q = (torch.rand((8, N), generator=g, dtype=torch.float64) * 4 - 2).to(dev)
    ids = [j.id for j in arm]
    hp, ht = m.find_joint("head_pan_joint"), m.find_joint("head_tilt_joint")

    def check(extra=()):
        om = _oracle_with(tree, {hp.id: m.joint_angle(hp), ht.id: m.joint_angle(ht)}, extra)
        P = kinhip.get_transform_batch(m, links, arm, Q).cpu().numpy()
        ref = om.fk_batch(Q.cpu().numpy(), ids, [l.id for l in links])
        np.testing.assert_allclose(P, ref, atol=1e-12)
        pose, J = kinhip.get_jacobian_batch(m, gl, arm, Q)
        ps, js = om.fk_jac_batch(Q.cpu().numpy(), ids, gl.id, ids, True, False)
        np.testing.assert_allclose(pose.cpu().numpy(), ps, atol=1e-12)
        np.testing.assert_allclose(J.cpu().numpy(), js, atol=1e-12)
        return P

    p0 = check()
    assert np.array_equal(p0, check())  # cached plans: same results
    m.set_joint_angle(hp, 0.7)  # a joint the batch does not drive: the cached plans must be re-staged
    m.set_joint_angle(ht, -0.3)
    p1 = check()
    assert not np.array_equal(p0[1], p1[1]) and np.array_equal(p0[0], p1[0])  # head moved, gripper did not
    # add_new_link (src/mechanism.jl:238-267): a fixed child of gripper_link, then query it
    T = np.eye(4)
    T[:3, 3] = [0.05, -0.02, 0.1]
    nl = m.add_new_link(kinhip.Link("tool_tip"), gl, T)
    om = _oracle_with(tree, {hp.id: 0.7, ht.id: -0.3}, [(gl.id, T)])
    P = kinhip.get_transform_batch(m, [nl, gl], arm, Q).cpu().numpy()
    ref = om.fk_batch(Q.cpu().numpy(), ids, [nl.id, gl.id])
    np.testing.assert_allclose(P, ref, atol=1e-12)
    check(extra=[(gl.id, T)])  # the earlier requests still answer correctly after the tree grew


def test_oneshot_c_abi_errors(dev):
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    L = K.lib()
    Q = torch.zeros((8, 16), dtype=torch.float32, device=dev)
    ids = np.array([m.find_joint(n).id for n in ARM], np.int32)
    out = torch.empty((1, 12, 16), dtype=torch.float32, device=dev)
    bad = np.array([999], np.int32)
    rc = L.kin_get_transform_batch(m._model, K.KIN_F32, 8, ids.ctypes.data_as(C.c_void_p), Q.data_ptr(), 16, 16, 1,
                                   bad.ctypes.data_as(C.c_void_p), out.data_ptr(), 16, None)
    assert rc == K.KIN_E_KEY  # unknown link id: Julia's KeyError
    with pytest.raises(KeyError):
        kinhip.get_jacobian_batch(m, kinhip.Link("nope", id=999), [m.find_joint(n) for n in ARM], Q.double())


def test_host_tensors_are_refused_before_the_kernel(dev):
    """A CPU (or other-device) tensor next to a device Q raises in Python, never reaches a kernel."""
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32)
    Q = torch.zeros((8, 64), dtype=torch.float32, device=dev)
    with pytest.raises(ValueError):
        plan.ik_dls(torch.zeros((12, 64), dtype=torch.float32), Q)  # host targets
    with pytest.raises(ValueError):
        plan.run(Q, poses=torch.empty((1, 12, 64), dtype=torch.float32))  # host output
    pn = m.plan(arm, jac_link=gl, jac_joints=arm, with_rot=False, dtype=torch.float32)
    with pytest.raises(ValueError):
        pn.point_ik_nakamura(torch.zeros((3, 64), dtype=torch.float32), Q)
    with pytest.raises(ValueError):
        kinhip.get_transform_batch(m, [gl], arm, Q, poses=torch.empty((1, 12, 64), dtype=torch.float32))
    sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
    sdf = kinhip.UnionSDF([kinhip.BoxSDF(np.eye(4), (0.1, 0.1, 0.1))])
    cp = sscc.plan(arm, dtype=torch.float32)
    with pytest.raises(ValueError):
        cp.run(sdf, Q, dists=torch.empty((cp.n_sph, 64), dtype=torch.float32))
    torch.cuda.synchronize()
