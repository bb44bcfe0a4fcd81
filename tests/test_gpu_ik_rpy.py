"""The reference's IK objective in the batched DLS kernel (kin_ik_params.with_rot = 2):
f_objective of src/inverse_kinematics.jl:38-50 minimises |[p* - p; rpy(target) - rpy(pose)]|^2 with
the rpy_jac=true Jacobian (src/algorithm.jl:56-63, 83-106).  The kernel takes damped Gauss-Newton
steps on exactly that residual (angle differences wrapped to (-pi, pi]) and stops when |dp| and
|d rpy| are below tol_pos / tol_rot -- the reference test's metric (test/test_inverse_kinematics.jl:
19-23: |d rpy| and |dp| <= 1e-3).

  * fp64 iterates equal the oracle restatement (or_ik_dls_batch with with_rot = 2): the same
    iteration counts, angles within 1e-7, generic and plan-specialised kernels, with and without base;
  * acceptance in the reference's metric at EVERY pitch, including the near-gimbal targets
    (|cos pitch| <= 0.2) that the axis-angle test (tests/test_gpu_parity.py::test_ik_dls_acceptance)
    cannot judge in rpy; fp32 and fp64, the bench's solver settings."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import ARM, golden

import kinhip

pytestmark = pytest.mark.gpu

KW = dict(max_iters=64, restarts=3, seed=0, lam=1e-2, max_step=0.5, tol_pos=1e-3, tol_rot=1e-3)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda", 0)


def _targets(om, ids, link, N, seed, arm, with_base=False):
    lo = np.nan_to_num(np.array([j.lower_limit for j in arm]), neginf=-np.pi)
    hi = np.nan_to_num(np.array([j.upper_limit for j in arm]), posinf=np.pi)
    rng = np.random.default_rng(seed)
    q = lo[:, None] + (hi - lo)[:, None] * rng.random((len(arm), N))
    if with_base:
        q = np.vstack([q, rng.uniform(-0.5, 0.5, (3, N))])
    return om.fk_batch(q, ids, [link])[0]


def _pitch_cos(tgt):
    """|cos(pitch)| of 3x4 column-major poses [12, N] (RotZYX: pitch = -asin(R31))."""
    return np.sqrt(np.maximum(0.0, 1.0 - tgt[2] ** 2))


@pytest.mark.parametrize("spec", [False, True])
@pytest.mark.parametrize("with_base", [False, True])
def test_rpy_objective_iterates_vs_oracle(dev, spec, with_base):
    m = kinhip.parse_urdf(golden("fetch.urdf"), with_base=with_base)
    arm = [m.find_joint(n) for n in ARM]
    gl = m.find_link("gripper_link")
    tree = O.parse_urdf_tree(golden("fetch.urdf"))
    om = O.OracleMech(tree, with_base=with_base)
    ids = [j.id for j in arm]
    N = 1000
    tgt = _targets(om, ids, gl.id, N, 41 + with_base, arm, with_base)
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float64)
    if spec:
        plan.specialize(kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
    nq = 8 + (3 if with_base else 0)
    Q, it, err = plan.ik_dls(torch.tensor(tgt, device=dev).contiguous(), torch.zeros((nq, N), dtype=torch.float64,
                                                                                  device=dev), with_rot=2, **KW)
    rq, rit, rerr = om.ik_dls_batch(np.zeros((nq, N)), ids, gl.id, tgt, with_rot=2, **KW)
    it = it.cpu().numpy()
    assert (it <= 64).mean() >= 0.99
    np.testing.assert_array_equal(it, rit)
    np.testing.assert_allclose(Q.cpu().numpy(), rq, atol=1e-7)
    np.testing.assert_allclose(err.cpu().numpy(), rerr, atol=1e-9)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_rpy_objective_acceptance_at_every_pitch(dev, dtype):
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    gl = m.find_link("gripper_link")
    om = O.OracleMech(O.parse_urdf_tree(golden("fetch.urdf")))
    ids = [j.id for j in arm]
    tgt = _targets(om, ids, gl.id, 16384, 7, arm)
    cp = _pitch_cos(tgt)
    near = np.nonzero(cp <= 0.2)[0]
    assert near.size >= 200  # enough near-gimbal targets in the sample
    # the whole sample plus the near-gimbal ones again as their own batch
    for sel in (np.arange(tgt.shape[1]), near):
        T = tgt[:, sel]
        n = T.shape[1]
        plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype).specialize(kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
        Q, it, err = plan.ik_dls(torch.tensor(T, dtype=dtype, device=dev).contiguous(),
                                 torch.zeros((8, n), dtype=dtype, device=dev), with_rot=2, **KW)
        conv = it.cpu().numpy() <= 64
        assert conv.mean() >= 0.99, (n, conv.mean())
        q = Q.double().cpu().numpy()
        got = om.fk_batch(q, ids, [gl.id])[0]
        # the reference's metric, recomputed by the oracle's FK at the returned angles
        dp = np.linalg.norm(got[9:] - T[9:], axis=0)
        drpy = np.zeros((3, n))
        for k in range(n):
            Ta, Tt = np.eye(4), np.eye(4)
            Ta[:3, :4] = got[:, k].reshape(4, 3).T
            Tt[:3, :4] = T[:, k].reshape(4, 3).T
            d = O.rpy(Ta) - O.rpy(Tt)
            drpy[:, k] = (d + np.pi) % (2 * np.pi) - np.pi
        assert np.all(dp[conv] < 1e-3)
        assert np.all(np.abs(drpy[:, conv]) < 1e-3), float(np.abs(drpy[:, conv]).max())
        lo = np.array([j.lower_limit for j in arm])
        hi = np.array([j.upper_limit for j in arm])
        tol = 1e-6 if dtype == torch.float32 else 0
        assert np.all(q >= lo[:, None] - tol) and np.all(q <= hi[:, None] + tol)


def test_with_rot_out_of_range_is_refused(dev):
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32)
    with pytest.raises(kinhip.KinError):
        plan.ik_dls(torch.zeros((12, 4), dtype=torch.float32, device=dev), torch.zeros((8, 4), dtype=torch.float32,
                                                                                     device=dev), with_rot=3)
