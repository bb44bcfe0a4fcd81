"""GPU parity: the HIP engine (through the C-ABI) vs the CPU oracle and the golden fixtures.

Tolerances (stated per BASELINE north star: poses / Jacobian entries within 1e-6 absolute):
  fp64 kernels: 1e-9 absolute vs the oracle (observed ~1e-15)
  fp32 kernels: 1e-6 absolute vs the oracle evaluated at the fp32-rounded angles (the north star;
    observed ~4e-7).  Angles here are drawn in [-2.5, 2.5], beyond some limits; rpy-Jacobian rows
    (which divide by cos(pitch)) get 20x.  tests/test_gpu_fp32_gate.py gates the bench's exact path.
"""
import json

import numpy as np
import pytest
import torch

import oracle as O
from conftest import ARM, EXAMPLE_LINKS, golden

import kinhip

pytestmark = pytest.mark.gpu

TOL = {torch.float64: 1e-9, torch.float32: 1e-6}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def fetch_tree():
    return O.parse_urdf_tree(golden("fetch.urdf"))


def _fetch(with_base=False):
    m = kinhip.parse_urdf(golden("fetch.urdf"), with_base=with_base)
    return m, [m.find_joint(n) for n in ARM]


def _rand_q(n, ncol, seed, dtype, dev, lo=-2.5, hi=2.5):
    g = torch.Generator().manual_seed(seed)
    q = torch.rand((ncol, n), generator=g, dtype=torch.float64) * (hi - lo) + lo
    return q.to(dtype).to(dev)


# ---------------------------------------------------------------- fixtures ---
@pytest.mark.parametrize("with_base", [False, True])
def test_ground_truth_json_on_gpu(dev, with_base):
    """test/test_kinematics.jl:10-41 through the GPU (PR2 fragment, fp64), all 9 links, twice."""
    gt = json.load(open(golden("ground_truth.json")))
    m = kinhip.parse_urdf(golden("pr2_torso_rarm.urdf"), with_base=with_base)
    joints = [m.find_joint(n) for n in gt["joint_names"]]
    links = [m.find_link(n) for n in gt["link_names"]]
    angles = list(gt["angle_vector"]) + ([0.3, 0.3, 0.3] if with_base else [])
    Q = torch.tensor(angles, dtype=torch.float64, device=dev).reshape(-1, 1).repeat(1, 3).contiguous()
    poses = kinhip.get_transform_batch(m, links, joints, Q).cpu().numpy()
    # the same request through a plan-specialised kernel (constants of the PR2 fragment folded)
    ps = m.plan(joints, out_links=links, dtype=torch.float64).specialize(kinhip.KIN_SPEC_FK).run(Q)[0]
    np.testing.assert_array_equal(ps.cpu().numpy(), poses)
    th = 0.3
    Rz = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
    for rep in range(2):
        for k, pg in enumerate(gt["pose_list"]):
            T = np.eye(4)
            T[:3, :4] = poses[k, :, rep].reshape(4, 3).T
            r = kinhip.rpy(T)
            ypr = np.array([r[2], r[1], r[0]])
            pg = np.asarray(pg)
            if with_base:
                np.testing.assert_allclose(T[:3, 3], Rz @ pg[:3] + [0.3, 0.3, 0], atol=1e-6)
                np.testing.assert_allclose(ypr, pg[3:] + [0.3, 0, 0], atol=1e-6)
            else:
                np.testing.assert_allclose(T[:3, 3], pg[:3], atol=1e-6)
                np.testing.assert_allclose(ypr, pg[3:], atol=1e-6)
    # and the single-configuration API (get_transform) on the same fixture
    m.set_joint_angles(joints, angles)
    T = kinhip.get_transform(m, links[5])
    ref = np.asarray(gt["pose_list"][5])
    if not with_base:
        np.testing.assert_allclose(T[:3, 3], ref[:3], atol=1e-9)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_golden_fetch_fixture(dev, dtype):
    g = np.load(golden("fetch_fk_jac_golden.npz"))
    m, arm = _fetch()
    Q = torch.tensor(g["q"], dtype=dtype, device=dev).contiguous()
    tol = 1e-9 if dtype == torch.float64 else 5e-5  # fp32: fixture angles are fp64 (not re-rounded)
    poses = kinhip.get_transform_batch(m, m.links, arm, Q).double().cpu().numpy()
    np.testing.assert_allclose(poses, g["poses"], atol=tol)
    gl = m.find_link("gripper_link")
    pose, jac = kinhip.get_jacobian_batch(m, gl, arm, Q, with_rot=True)
    np.testing.assert_allclose(jac.double().cpu().numpy(), g["jac_geo"], atol=tol)
    np.testing.assert_allclose(pose.double().cpu().numpy(), g["poses"][gl.id - 1], atol=tol)
    # the bench's path: specialised plan, tiled layout, against the same golden vectors
    sp = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype).specialize(kinhip.KIN_SPEC_FK)
    Pt, Jt = sp.run_tiled(kinhip.tiled(Q, 256), Q.shape[1])
    np.testing.assert_allclose(kinhip.untiled(Jt, Q.shape[1]).double().cpu().numpy(), g["jac_geo"], atol=tol)
    np.testing.assert_allclose(kinhip.untiled(Pt, Q.shape[1])[0].double().cpu().numpy(), g["poses"][gl.id - 1],
                               atol=tol)
    _, jr = kinhip.get_jacobian_batch(m, gl, arm, Q, with_rot=True, rpy_jac=True)
    jr = jr.double().cpu().numpy()
    ok = np.abs(np.cos(np.arcsin(np.clip(-g["poses"][gl.id - 1][2], -1, 1)))) > 1e-2  # away from pitch = +-pi/2
    np.testing.assert_allclose(jr[:, :, ok], g["jac_rpy"][:, :, ok], atol=tol * 10)
    mb, armb = _fetch(with_base=True)
    Qb = torch.tensor(g["qb"], dtype=dtype, device=dev).contiguous()
    pb, jb = kinhip.get_jacobian_batch(mb, mb.find_link("gripper_link"), armb, Qb)
    np.testing.assert_allclose(pb.double().cpu().numpy(), g["pose_base"], atol=tol)
    np.testing.assert_allclose(jb.double().cpu().numpy(), g["jac_base"], atol=tol)


# ------------------------------------------------------------ vs oracle ------
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("with_base", [False, True])
@pytest.mark.parametrize("rpy_jac", [False, True])
def test_fk_jac_vs_oracle(dev, fetch_tree, dtype, with_base, rpy_jac):
    m, arm = _fetch(with_base)
    N = 3000  # not a multiple of the block size
    Q = _rand_q(N, 8 + (3 if with_base else 0), 7, dtype, dev)
    gl = m.find_link("gripper_link")
    pose, jac = kinhip.get_jacobian_batch(m, gl, arm, Q, with_rot=True, rpy_jac=rpy_jac)
    om = O.OracleMech(fetch_tree, with_base=with_base)
    qd = Q.double().cpu().numpy()
    ps, js = om.fk_jac_batch(qd, [j.id for j in arm], gl.id, [j.id for j in arm], True, rpy_jac)
    np.testing.assert_allclose(pose.double().cpu().numpy(), ps, atol=TOL[dtype])
    jg = jac.double().cpu().numpy()
    if rpy_jac:  # rpy rows blow up at pitch = +-pi/2; compare where cos(pitch) is not tiny
        c = np.sqrt(ps[0] ** 2 + ps[1] ** 2)  # cos(pitch)
        ok = c > 0.05
        np.testing.assert_allclose(jg[:, :3], js[:, :3], atol=TOL[dtype])
        # rpy rates: the ZYX rate map carries 1/cos(pitch) and its rounding 1/cos^2 (<= 400x here)
        err = np.abs(jg[:, 3:, ok] - js[:, 3:, ok])
        assert np.all(err <= TOL[dtype] / c[ok] ** 2), float((err * c[ok] ** 2).max())
    else:
        np.testing.assert_allclose(jg, js, atol=TOL[dtype])


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_multi_link_fk_vs_oracle(dev, fetch_tree, dtype):
    """Config 2 shape (exampel.jl:11 links) and every link, with LDS branch slots."""
    m, arm = _fetch()
    Q = _rand_q(2049, 8, 11, dtype, dev)
    om = O.OracleMech(fetch_tree)
    for names in (EXAMPLE_LINKS, [l.name for l in m.links], ["r_gripper_finger_link", "head_pan_link", "base_link",
                                                                "laser_link", "l_gripper_finger_link"]):
        links = [m.find_link(n) for n in names]
        poses = kinhip.get_transform_batch(m, links, arm, Q).double().cpu().numpy()
        ref = om.fk_batch(Q.double().cpu().numpy(), [j.id for j in arm], [l.id for l in links])
        np.testing.assert_allclose(poses, ref, atol=TOL[dtype])


def test_jacobian_column_semantics(dev, fetch_tree):
    """get_jacobian! (untouched) vs get_jacobian (zeros), irrelevant and repeated columns,
    q joints != Jacobian joints, non-batched joints at m.angles (src/algorithm.jl:83-114)."""
    m, arm = _fetch()
    head = m.find_joint("head_pan_joint")
    jj = [arm[3], head, arm[0], arm[3], arm[6]]  # repeated column, irrelevant head column
    gl = m.find_link("gripper_link")
    qj = arm[:5]  # joints 6..8 stay at m.angles
    defaults = np.zeros(len(m.joints))
    for j, a in zip(arm[5:], [0.4, -0.7, 1.1]):
        defaults[j.id - 1] = a
    m.angles[:] = defaults
    m._angles_synced = False
    N = 700
    Q = _rand_q(N, 5, 3, torch.float64, dev)
    om = O.OracleMech(fetch_tree)
    om_ids = [j.id for j in qj] + [j.id for j in arm[5:]]
    qfull = np.vstack([Q.cpu().numpy(), np.tile(np.array([[0.4], [-0.7], [1.1]]), (1, N))])
    for zero in (True, False):
        plan = m.plan(qj, out_links=[gl], jac_link=gl, jac_joints=jj, zero_fill=zero, dtype=torch.float64)
        init = torch.full((len(jj), 6, N), 9.0, dtype=torch.float64, device=dev)
        _, jac = plan.run(Q, jac=init)
        init_np = np.full((len(jj), 6, N), 9.0)
        _, ref = om.fk_jac_batch(qfull, om_ids, gl.id, [j.id for j in jj], True, False, zero_fill=zero,
                                 jac_init=init_np)
        np.testing.assert_allclose(jac.cpu().numpy(), ref, atol=1e-9)
        if not zero:
            assert np.all(jac.cpu().numpy()[1] == 9.0)       # head column untouched
            assert np.all(jac.cpu().numpy()[2, 3:] == 9.0)   # prismatic torso: rows 4:6 untouched


def test_fd_jacobian_on_gpu(dev):
    """Analytic GPU Jacobian vs forward differences of GPU FK (test_kinematics.jl:57-66)."""
    m, arm = _fetch(with_base=True)
    gl = m.find_link("gripper_link")
    N = 256
    Q = _rand_q(N, 11, 5, torch.float64, dev, -1.5, 1.5)
    pose, jac = kinhip.get_jacobian_batch(m, gl, arm, Q, with_rot=True)
    eps = 1e-7
    for c in range(11):
        Q1 = Q.clone()
        Q1[c] += eps
        p1 = kinhip.get_transform_batch(m, [gl], arm, Q1)[0]
        fd = (p1[9:12] - pose[9:12]) / eps
        torch.testing.assert_close(fd, jac[c, :3], atol=1e-5, rtol=0)


def test_edge_sizes_and_strides(dev, fetch_tree):
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float64)
    om = O.OracleMech(fetch_tree)
    for N in (1, 63, 64, 65, 257):
        Q = _rand_q(N, 8, N, torch.float64, dev)
        poses, jac = plan.run(Q)
        ps, js = om.fk_jac_batch(Q.cpu().numpy(), [j.id for j in arm], gl.id, [j.id for j in arm])
        np.testing.assert_allclose(poses[0].cpu().numpy(), ps, atol=1e-9)
        np.testing.assert_allclose(jac.cpu().numpy(), js, atol=1e-9)
    # ldq > N: a column-padded Julia matrix view
    big = _rand_q(300, 8, 1, torch.float64, dev)
    Qv = big[:, :200]
    poses, _ = plan.run(Qv)
    ps, _ = om.fk_jac_batch(Qv.cpu().numpy(), [j.id for j in arm], gl.id, [j.id for j in arm])
    np.testing.assert_allclose(poses[0].cpu().numpy(), ps, atol=1e-9)
    # N = 0 is a no-op
    plan.run(torch.empty((8, 0), dtype=torch.float64, device=dev))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("with_base", [False, True])
def test_tiled_layout(dev, fetch_tree, dtype, with_base):
    """kin_plan_run_tiled: (ntiles, rows, tile) layout == plain SoA bit for bit, and vs the oracle;
    partial last tile, one tile, row padding inside a tile, phase-B links."""
    m, arm = _fetch(with_base)
    gl = m.find_link("gripper_link")
    links = [gl] + [m.find_link(n) for n in EXAMPLE_LINKS]
    plan = m.plan(arm, out_links=links, jac_link=gl, dtype=dtype)
    om = O.OracleMech(fetch_tree, with_base=with_base)
    for N, tile in ((3000, 256), (5000, 1024), (700, 1024), (4096, 4096)):
        Q = _rand_q(N, plan.n_qcols, N + tile, dtype, dev)
        P0, J0 = plan.run(Q)
        Pt, Jt = plan.run_tiled(kinhip.tiled(Q, tile), N)
        assert torch.equal(kinhip.untiled(Pt, N), P0) and torch.equal(kinhip.untiled(Jt, N), J0)
        ps, js = om.fk_jac_batch(Q.double().cpu().numpy(), [j.id for j in arm], gl.id, [j.id for j in arm])
        np.testing.assert_allclose(kinhip.untiled(Jt, N).double().cpu().numpy(), js, atol=TOL[dtype])
        np.testing.assert_allclose(kinhip.untiled(Pt, N)[0].double().cpu().numpy(), ps, atol=TOL[dtype])
    # rows padded inside each tile (ld > tile) and tiles padded apart (ts > rows * ld)
    N, tile = 2000, 512
    Q = _rand_q(N, plan.n_qcols, 1, dtype, dev)
    nt = -(-N // tile)
    Qt = torch.zeros((nt, plan.n_qcols, tile + 64), dtype=dtype, device=dev)
    Qt[:, :, :tile] = kinhip.tiled(Q, tile)
    Pb = torch.full((nt + 1, len(links), 12, tile + 32), 7.0, dtype=dtype, device=dev)
    Jb = torch.full((nt, plan.jac_cols + 1, 6, tile + 96), 7.0, dtype=dtype, device=dev)
    Pv = Pb[:nt, :, :, :tile]
    Jv = Jb[:, :plan.jac_cols, :, :tile]
    plan.run_tiled(Qt[:, :, :tile], N, poses=Pv, jac=Jv)
    P0, J0 = plan.run(Q)
    assert torch.equal(kinhip.untiled(Pv.contiguous(), N), P0)
    assert torch.equal(kinhip.untiled(Jv.contiguous(), N), J0)
    assert bool((Pb[nt] == 7.0).all()) and bool((Jb[:, plan.jac_cols] == 7.0).all())
    assert bool((Pb[..., tile:] == 7.0).all()) and bool((Jb[..., tile:] == 7.0).all())
    # bad tilings are refused, never launched
    with pytest.raises(kinhip.KinError):
        plan.run_tiled(torch.zeros((2, plan.n_qcols, 100), dtype=dtype, device=dev), 200)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("with_base", [False, True])
@pytest.mark.parametrize("rpy_jac", [False, True])
def test_specialized_fk_equals_generic(dev, fetch_tree, dtype, with_base, rpy_jac):
    """kin_plan_specialize: the constant-folded kernel gives the generic kernel's results (values
    equal; only the sign of a zero may differ) for FK + J, phase-B links, plain and tiled layouts."""
    m, arm = _fetch(with_base)
    gl = m.find_link("gripper_link")
    links = [gl] + [m.find_link(n) for n in EXAMPLE_LINKS] + [m.find_link("head_camera_rgb_optical_frame")]
    N = 3001
    Q = _rand_q(N, 8 + (3 if with_base else 0), 17, dtype, dev)
    gen = m.plan(arm, out_links=links, jac_link=gl, rpy_jac=rpy_jac, dtype=dtype)
    spe = m.plan(arm, out_links=links, jac_link=gl, rpy_jac=rpy_jac, dtype=dtype)
    assert spe.specialized == 0
    spe.specialize(kinhip.KIN_SPEC_FK)
    assert spe.specialized == kinhip.KIN_SPEC_FK
    spe.specialize()  # every kind that applies (+ IK without rpy rows) keeps FK
    assert spe.specialized & kinhip.KIN_SPEC_FK
    assert bool(spe.specialized & kinhip.KIN_SPEC_IK) == (not rpy_jac)
    P0, J0 = gen.run(Q)
    P1, J1 = spe.run(Q)
    assert torch.equal(P0, P1) and torch.equal(J0, J1)
    Pt, Jt = spe.run_tiled(kinhip.tiled(Q, 1024), N)
    assert torch.equal(kinhip.untiled(Pt, N), P0) and torch.equal(kinhip.untiled(Jt, N), J0)
    om = O.OracleMech(fetch_tree, with_base=with_base)
    ps, js = om.fk_jac_batch(Q.double().cpu().numpy(), [j.id for j in arm], gl.id, [j.id for j in arm], True,
                             rpy_jac)
    np.testing.assert_allclose(P1[0].double().cpu().numpy(), ps, atol=TOL[dtype])


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("with_base", [False, True])
def test_specialized_strided_large_batch(dev, with_base, dt):
    """Batches of >= 2^23 configurations (which rounds 2-5 ran on a grid-strided specialised k_fk; since round 6
    the one-per-lane grid at every size, the faster one in both precisions, profiles/r06_fk_stride_ab.txt; a
    launch chunk is 2^27): equal to the generic kernel on plain and tiled layouts, with a partial last unit and
    a partial last tile, and phase-B links in the plan."""
    m, arm = _fetch(with_base)
    gl = m.find_link("gripper_link")
    links = [gl, m.find_link("wrist_flex_link"), m.find_link("head_camera_rgb_optical_frame")]
    N = (1 << 23) + 1000
    Q = _rand_q(N, 8 + (3 if with_base else 0), 23, dt, dev)
    gen = m.plan(arm, out_links=links, jac_link=gl, dtype=dt)
    spe = m.plan(arm, out_links=links, jac_link=gl, dtype=dt).specialize(kinhip.KIN_SPEC_FK)
    P0, J0 = gen.run(Q)
    P1, J1 = spe.run(Q)
    assert torch.equal(P0, P1) and torch.equal(J0, J1)
    del P1, J1
    Pt, Jt = spe.run_tiled(kinhip.tiled(Q, 8192), N)
    assert torch.equal(kinhip.untiled(Pt, N), P0) and torch.equal(kinhip.untiled(Jt, N), J0)


def test_specialized_column_semantics(dev, fetch_tree):
    """Specialised plans honour m.angles of non-batched joints, repeated / irrelevant columns and
    get_jacobian! (untouched) vs get_jacobian (zeros) like the generic ones."""
    m, arm = _fetch()
    head = m.find_joint("head_pan_joint")
    jj = [arm[3], head, arm[0], arm[3], arm[6]]
    gl = m.find_link("gripper_link")
    qj = arm[:5]
    for j, a in zip(arm[5:], [0.4, -0.7, 1.1]):
        m.set_joint_angle(j, a)
    Q = _rand_q(700, 5, 3, torch.float64, dev)
    for zero in (True, False):
        gen = m.plan(qj, out_links=[gl], jac_link=gl, jac_joints=jj, zero_fill=zero, dtype=torch.float64)
        spe = m.plan(qj, out_links=[gl], jac_link=gl, jac_joints=jj, zero_fill=zero, dtype=torch.float64)
        spe.specialize(kinhip.KIN_SPEC_FK)
        a = torch.full((len(jj), 6, 700), 9.0, dtype=torch.float64, device=dev)
        b = a.clone()
        gen.run(Q, jac=a)
        spe.run(Q, jac=b)
        assert torch.equal(a, b)


def test_large_batch_properties(dev, fetch_tree):
    """BASELINE size (2^20, fp32): size-independent properties + a strided oracle sample."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    lo = [j.lower_limit for j in arm]
    hi = [j.upper_limit for j in arm]
    N = 1 << 20
    Q = kinhip.uniform_configs(lo, hi, N, dtype=torch.float32, device=dev)
    pose, jac = kinhip.get_jacobian_batch(m, gl, arm, Q)
    R = pose[:9].reshape(3, 3, N).permute(2, 1, 0)  # [N, row, col]
    eye = torch.eye(3, device=dev).expand(N, 3, 3)
    assert float((R @ R.transpose(1, 2) - eye).abs().max()) < 5e-6
    # angular rows of revolute columns are unit axes; torso (prismatic) linear rows too
    nrm = jac[1:, 3:].norm(dim=1)
    assert float((nrm - 1).abs().max()) < 1e-5
    assert float((jac[0, :3].norm(dim=0) - 1).abs().max()) < 1e-5
    # linear rows = z x (p - o) => orthogonal to z
    dot = (jac[1:, :3] * jac[1:, 3:]).sum(1)
    assert float(dot.abs().max()) < 1e-5
    idx = torch.arange(0, N, 4099, device=dev)
    om = O.OracleMech(fetch_tree)
    ps, js = om.fk_jac_batch(Q[:, idx].double().cpu().numpy(), [j.id for j in arm], gl.id, [j.id for j in arm])
    np.testing.assert_allclose(pose[:, idx].double().cpu().numpy(), ps, atol=2e-5)
    np.testing.assert_allclose(jac[:, :, idx].double().cpu().numpy(), js, atol=2e-5)


# -------------------------------------------------------------------- IK ------
def test_nakamura_vs_oracle(dev, fetch_tree):
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    N = 512
    plan = m.plan(arm, jac_link=gl, jac_joints=arm, with_rot=False, dtype=torch.float64)
    Q0 = _rand_q(N, 8, 2, torch.float64, dev, -0.5, 0.5)
    g = torch.Generator().manual_seed(3)
    pts = (torch.rand((3, N), generator=g, dtype=torch.float64) * torch.tensor([[0.6], [1.0], [0.8]])
           + torch.tensor([[0.3], [-0.5], [0.5]])).to(dev).contiguous()
    Q = plan.point_ik_nakamura(pts, Q0.clone())
    om = O.OracleMech(fetch_tree)
    ref = om.point_ik_nakamura_batch(Q0.cpu().numpy(), [j.id for j in arm], gl.id, pts.cpu().numpy())
    np.testing.assert_allclose(Q.cpu().numpy(), ref, atol=1e-7)
    # single-config API
    m.set_joint_angles(arm, np.zeros(8))
    q1 = kinhip.point_inverse_kinematics_nakamura(m, gl, arm, [0.7, 0.2, 0.9])
    r1 = O.OracleMech(fetch_tree).point_ik_nakamura(gl.id, [j.id for j in arm], [0.7, 0.2, 0.9])
    np.testing.assert_allclose(q1, r1, atol=1e-8)


def _targets(om, arm_ids, gl, N, seed, with_base=False):
    lo = np.array([om.tree.joint_lower[i - 1] for i in arm_ids])
    hi = np.array([om.tree.joint_upper[i - 1] for i in arm_ids])
    lo = np.where(np.isfinite(lo), lo, -np.pi)
    hi = np.where(np.isfinite(hi), hi, np.pi)
    rng = np.random.default_rng(seed)
    qt = lo[:, None] + (hi - lo)[:, None] * rng.random((len(arm_ids), N))
    if with_base:
        qt = np.vstack([qt, rng.uniform(-1, 1, (3, N))])
    return om.fk_batch(qt, arm_ids, [gl])[0]


def test_ik_dls_iterates_vs_oracle(dev, fetch_tree):
    """fp64 kernel == fp64 oracle restatement of the same DLS (short runs, iterate parity)."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    ids = [j.id for j in arm]
    om = O.OracleMech(fetch_tree)
    N = 512
    tgt = _targets(om, ids, gl.id, N, 4)
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float64)
    for iters in (1, 3, 8):
        Q = torch.zeros((8, N), dtype=torch.float64, device=dev)
        T = torch.tensor(tgt, device=dev).contiguous()
        Q, it, err = plan.ik_dls(T, Q, max_iters=iters)
        rq, rit, rerr = om.ik_dls_batch(np.zeros((8, N)), ids, gl.id, tgt, max_iters=iters)
        np.testing.assert_allclose(Q.cpu().numpy(), rq, atol=1e-7)
        np.testing.assert_array_equal(it.cpu().numpy(), rit)


@pytest.mark.parametrize("lanes", [0, 1, 2, 4, 8])
def test_ik_dls_restarts_vs_oracle(dev, fetch_tree, lanes):
    """Restart re-seeding (counter hash of seed, index, attempt, column) identical on both sides,
    whether the attempts run in one lane or side by side in 2/4/8 lanes of a target."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    ids = [j.id for j in arm]
    om = O.OracleMech(fetch_tree)
    N = 300
    tgt = _targets(om, ids, gl.id, N, 21)
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float64)
    Q = torch.zeros((8, N), dtype=torch.float64, device=dev)
    Q, it, err = plan.ik_dls(torch.tensor(tgt, device=dev).contiguous(), Q, max_iters=13, restarts=3, seed=77,
                             tol_pos=1e-12, tol_rot=1e-12, lanes=lanes)
    rq, rit, _ = om.ik_dls_batch(np.zeros((8, N)), ids, gl.id, tgt, max_iters=13, restarts=3, seed=77,
                                 tol_pos=1e-12, tol_rot=1e-12)
    np.testing.assert_array_equal(it.cpu().numpy(), rit)
    np.testing.assert_allclose(Q.cpu().numpy(), rq, atol=1e-7)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_ik_dls_lanes_identical(dev, fetch_tree, dtype):
    """Converging runs where the winning attempt varies by target: every lanes-per-target setting
    returns bit-identical angles, iteration counts and errors, and fp64 matches the oracle."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    ids = [j.id for j in arm]
    om = O.OracleMech(fetch_tree)
    N = 2000
    tgt = _targets(om, ids, gl.id, N, 33)
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype)
    T = torch.tensor(tgt, dtype=dtype, device=dev).contiguous()
    res = []
    for lanes in (1, 2, 4, 8):
        Q = torch.zeros((8, N), dtype=dtype, device=dev)
        res.append(plan.ik_dls(T, Q, max_iters=23, restarts=4, seed=5, lam=1e-2, max_step=0.5, lanes=lanes))
    it0 = res[0][1].cpu().numpy()
    assert len(set((it0 // 4).tolist())) > 2  # winners spread over several attempts (attempt length 4)
    for Q, it, err in res[1:]:
        assert torch.equal(Q, res[0][0]) and torch.equal(it, res[0][1]) and torch.equal(err, res[0][2])
    if dtype == torch.float64:
        rq, rit, _ = om.ik_dls_batch(np.zeros((8, N)), ids, gl.id, tgt, max_iters=23, restarts=4, seed=5)
        np.testing.assert_array_equal(it0, rit)
        np.testing.assert_allclose(res[0][0].cpu().numpy(), rq, atol=1e-7)


@pytest.mark.parametrize("dtype,damp_err", [(torch.float64, 0.0), (torch.float32, 0.0), (torch.float64, 0.01),
                                            (torch.float32, 0.01)])
def test_ik_dls_two_phase_identical(dev, fetch_tree, dtype, damp_err):
    """The two-phase schedule (automatic for this batch: 65,536 targets, 6 attempts of 4 iterations)
    returns the single-phase schedules' angles, iteration counts and errors bit for bit (lanes=1:
    sequential attempts, lanes=4: side by side), and fp64 matches the oracle on a subset."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    ids = [j.id for j in arm]
    om = O.OracleMech(fetch_tree)
    N = 1 << 16
    tgt = _targets(om, ids, gl.id, N, 57)
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype)
    if dtype == torch.float32:
        plan.specialize(kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
    T = torch.tensor(tgt, dtype=dtype, device=dev).contiguous()
    kw = dict(max_iters=23, restarts=4, seed=5, lam=1e-2, max_step=0.5, damp_err=damp_err)
    res = [plan.ik_dls(T, torch.zeros((8, N), dtype=dtype, device=dev), lanes=lanes, **kw) for lanes in (0, 1, 4)]
    it0 = res[0][1].cpu().numpy()
    assert len(set((it0 // 4).tolist())) > 3  # winners spread over several attempts: phase 2 does work
    for Q, it, err in res[1:]:
        assert torch.equal(Q, res[0][0]) and torch.equal(it, res[0][1]) and torch.equal(err, res[0][2])
    if dtype == torch.float64:
        k = 1000
        rq, rit, _ = om.ik_dls_batch(np.zeros((8, k)), ids, gl.id, tgt[:, :k], **kw)
        np.testing.assert_array_equal(it0[:k], rit)
        np.testing.assert_allclose(res[0][0][:, :k].cpu().numpy(), rq, atol=1e-7)


@pytest.mark.parametrize("damp_err,max_step", [(0.0, 0.5), (0.01, 1.0)])
def test_ik_dls_spec_two_phase_fp64_vs_oracle(dev, fetch_tree, damp_err, max_step):
    """Config 4's schedule in fp64 on the specialised kernels (two-phase with the hand-over; phase 2's
    lane-group minimum, ring prefix and ring lookup by DPP / v_readlane): bit-identical to the one-phase
    schedules of the same compilation (lanes 1 and 4) and to itself over repeated calls (the rings'
    control words carry over), and the first 1,000 targets equal the oracle restatement (equal
    iteration counts, angles to 1e-7) -- with a fixed lambda and with the error-scaled damping
    (kin_ik_params.damp_err, config 4's bench setting)."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    ids = [j.id for j in arm]
    om = O.OracleMech(fetch_tree)
    N = 1 << 16
    tgt = _targets(om, ids, gl.id, N, 58)
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float64)
    plan.specialize(kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
    T = torch.tensor(tgt, dtype=torch.float64, device=dev).contiguous()
    kw = dict(max_iters=64, restarts=3, seed=7, lam=1e-2, max_step=max_step, damp_err=damp_err)
    Z = torch.zeros((8, N), dtype=torch.float64, device=dev)
    ref = plan.ik_dls(T, Z.clone(), lanes=0, **kw)
    assert (ref[1] > 16).any()  # phase 2 did work
    for lanes in (0, 0, 1, 4):
        out = plan.ik_dls(T, Z.clone(), lanes=lanes, **kw)
        assert all(torch.equal(a, b) for a, b in zip(out, ref)), lanes
    k = 1000
    rq, rit, _ = om.ik_dls_batch(np.zeros((8, k)), ids, gl.id, tgt[:, :k], **kw)
    np.testing.assert_array_equal(ref[1][:k].cpu().numpy(), rit)
    np.testing.assert_allclose(ref[0][:, :k].cpu().numpy(), rq, atol=1e-7)


@pytest.mark.parametrize("dtype,N,lanes", [(torch.float32, 1 << 16, 0), (torch.float64, 1 << 16, 0),
                                             (torch.float32, 3000, 4), (torch.float64, 3000, 1)])
def test_ik_dls_from_q0_identical(dev, dtype, N, lanes):
    """kin_ik_dls_batch_from (starting angles read from Q0, Q written without being read) returns the
    in-place call's angles, iteration counts and errors bit for bit -- two-phase (65,536 targets) and
    one-phase schedules -- leaves Q0 unchanged, and q0 == q is the in-place call."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype)
    plan.specialize(kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
    lo, hi = [j.lower_limit for j in arm], [j.upper_limit for j in arm]
    T = plan.run(kinhip.uniform_configs(lo, hi, N, seed=31, dtype=dtype, device=dev))[0][0].contiguous()
    Q0 = kinhip.uniform_configs(lo, hi, N, seed=32, dtype=dtype, device=dev) * 0.5
    keep = Q0.clone()
    kw = dict(max_iters=64, restarts=3, seed=4, lam=1e-2, max_step=0.5, lanes=lanes)
    ref = plan.ik_dls(T, Q0.clone(), **kw)
    out = plan.ik_dls(T, torch.full_like(Q0, float("nan")), Q0=Q0, **kw)
    torch.cuda.synchronize()
    assert torch.equal(Q0, keep)
    for a, b in zip(out, ref):
        assert torch.equal(a, b)
    Qs = Q0.clone()
    same = plan.ik_dls(T, Qs, Q0=Qs, **kw)  # q0 == q: in place
    for a, b in zip(same, ref):
        assert torch.equal(a, b)
    with pytest.raises(ValueError):
        plan.ik_dls(T, torch.empty((8, N + 1), dtype=dtype, device=dev), Q0=Q0, **kw)


def test_ik_dls_two_phase_graph_replay(dev):
    """The two-phase schedule's scratch is a ring whose control words carry over between calls (no
    reset launch): a hipGraph captured around one call replays it any number of times, interleaved
    with eager calls of the same plan on the same stream, with the eager call's results bit for bit."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32)
    plan.specialize(kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
    N = 1 << 16
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, seed=91,
                                dtype=torch.float32, device=dev)
    T = plan.run(Qt)[0][0].contiguous()
    kw = dict(max_iters=64, restarts=3, seed=9, lam=1e-2, max_step=0.5)
    Q0 = torch.zeros((8, N), dtype=torch.float32, device=dev)
    ref = plan.ik_dls(T, Q0.clone(), **kw)  # eager; also allocates the plan's scratch before capture
    ref = [t.clone() for t in ref]
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    Qg = Q0.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            Qg.copy_(Q0)
            out = plan.ik_dls(T, Qg, stream=s, **kw)
        for rep in range(3):
            g.replay()
            s.synchronize()
            assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1]) and torch.equal(out[2], ref[2]), rep
            e = plan.ik_dls(T, Q0.clone(), stream=s, **kw)  # eager calls rotate through the other sets
            s.synchronize()
            assert torch.equal(e[0], ref[0]) and torch.equal(e[1], ref[1]), rep


def test_ik_dls_capture_first_call(dev):
    """a plan's first call that does not run the two-phase schedule (lanes = 4 with
    restarts, or a one-round batch) allocates nothing, so it may be the first call inside a stream
    capture; a first two-phase call inside a capture is refused with a message (it must allocate);
    several graphs of one plan each own a scratch set and replay the eager results bit for bit."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32)
    plan.specialize(kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
    N = 1 << 16
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, seed=93,
                                dtype=torch.float32, device=dev)
    T = plan.run(Qt)[0][0].contiguous()
    torch.cuda.synchronize()
    kw = dict(max_iters=64, restarts=3, seed=9, lam=1e-2, max_step=0.5)
    Q0 = torch.zeros((8, N), dtype=torch.float32, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        # first call of the plan, inside a capture, one-phase (lanes = 4): no allocation
        Qa = Q0.clone()
        ga = torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga, stream=s):
            outa = plan.ik_dls(T, Qa, stream=s, lanes=4, Q0=Q0, **kw)
        ga.replay()
        ga.replay()
        s.synchronize()
        refa = plan.ik_dls(T, Q0.clone(), stream=s, lanes=4, **kw)
        s.synchronize()
        assert torch.equal(outa[0], refa[0]) and torch.equal(outa[1], refa[1])
        # first two-phase call inside a capture: refused (it would allocate the scratch)
        gb = torch.cuda.CUDAGraph()
        with pytest.raises(kinhip.KinError, match="capture"):
            with torch.cuda.graph(gb, stream=s):
                plan.ik_dls(T, Q0.clone(), stream=s, **kw)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        ref = [t.clone() for t in plan.ik_dls(T, Q0.clone(), stream=s, **kw)]  # eager: allocates
        s.synchronize()
        graphs = []
        for k in range(6):  # 4 graphs own a set each, the 5th and 6th run one phase
            Qg = Q0.clone()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                out = plan.ik_dls(T, Qg, stream=s, Q0=Q0, **kw)  # seeds read from Q0: replays repeat
            graphs.append((g, out))
        for rep in range(2):
            for g, out in graphs:
                g.replay()
            e = plan.ik_dls(T, Q0.clone(), stream=s, **kw)
            s.synchronize()
            for g, out in graphs:
                assert all(torch.equal(a, b) for a, b in zip(out, ref)), rep
            assert all(torch.equal(a, b) for a, b in zip(e, ref)), rep


def test_plan_refuses_tensors_of_another_device(dev):
    """the Python mirror compares the tensors' device with the plan's (the C check only
    sees the current device)."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32)
    Q = torch.zeros((8, 64), dtype=torch.float32, device=dev)
    plan.run(Q)
    plan.device_index = dev.index + 1  # as if staged on another GPU
    with pytest.raises(ValueError, match="lives on"):
        plan.run(Q)
    with pytest.raises(ValueError, match="lives on"):
        plan.ik_dls(torch.zeros((12, 64), dtype=torch.float32, device=dev), Q)
    sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
    sdf = kinhip.UnionSDF([kinhip.BoxSDF(np.eye(4), (0.1, 0.1, 0.1))])
    cp = sscc.plan(arm, dtype=torch.float32)
    cp.run(sdf, Q)
    sdf.device_index = dev.index + 1
    with pytest.raises(ValueError, match="lives on"):
        cp.run(sdf, Q)
    torch.cuda.synchronize()


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_ik_dls_two_phase_large_identical(dev, dtype):
    """A batch of more than two rounds of resident waves (2^19 targets): phase 1 may run on wave-local
    queues (automatic where that does not lower the kernel's occupancy -- fp64 here, not fp32);
    angles, iteration counts and errors equal the one-phase schedule (lanes=4) bit for bit."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype)
    plan.specialize()
    N = 1 << 19
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, seed=77,
                                dtype=dtype, device=dev)
    T = plan.run(Qt)[0][0].contiguous()
    kw = dict(max_iters=64, restarts=3, seed=3, lam=1e-2, max_step=0.5)
    a = plan.ik_dls(T, torch.zeros((8, N), dtype=dtype, device=dev), lanes=0, **kw)
    b = plan.ik_dls(T, torch.zeros((8, N), dtype=dtype, device=dev), lanes=4, **kw)
    assert (a[1] > 16).any() and (a[1] <= 64).float().mean() > 0.99  # phase 2 did work; solves converge
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])


def test_ik_dls_two_phase_chunked_identical(dev):
    """A batch larger than the two-phase scratch list (2^20 + 5,000 targets) runs the two-phase schedule chunk
    by chunk (ik_chunk: 2^20 and 5,000), phase 1 of the fp32 kernel on the plain grid; angles, iteration counts
    and errors equal the one-phase schedule (lanes=4) bit for bit."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32)
    plan.specialize()
    N = (1 << 20) + 5000
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, seed=78,
                                dtype=torch.float32, device=dev)
    T = plan.run(Qt)[0][0].contiguous()
    del Qt
    kw = dict(max_iters=64, restarts=3, seed=5, lam=1e-2, max_step=0.5)
    a = plan.ik_dls(T, torch.zeros((8, N), dtype=torch.float32, device=dev), lanes=0, **kw)
    b = plan.ik_dls(T, torch.zeros((8, N), dtype=torch.float32, device=dev), lanes=4, **kw)
    assert (a[1] > 16).any() and (a[1] <= 64).float().mean() > 0.99
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])


def test_ik_dls_work_queue_identical(dev, fetch_tree):
    """Large batches run as per-wave work queues (a lane group that finishes takes the wave's next
    target): bit-identical to one target per group (lanes=1 here never queues), and the first
    targets match the oracle."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    ids = [j.id for j in arm]
    om = O.OracleMech(fetch_tree)
    N = 1 << 17
    tgt = _targets(om, ids, gl.id, N, 41)
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float64)
    T = torch.tensor(tgt, device=dev).contiguous()
    kw = dict(max_iters=32, restarts=3, seed=9)
    a = plan.ik_dls(T, torch.zeros((8, N), dtype=torch.float64, device=dev), lanes=4, **kw)
    b = plan.ik_dls(T, torch.zeros((8, N), dtype=torch.float64, device=dev), lanes=1, **kw)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    k = 1500
    rq, rit, _ = om.ik_dls_batch(np.zeros((8, k)), ids, gl.id, tgt[:, :k], **kw)
    np.testing.assert_array_equal(a[1][:k].cpu().numpy(), rit)
    np.testing.assert_allclose(a[0][:, :k].cpu().numpy(), rq, atol=1e-7)


def test_ik_dls_bench_config_slices_identical(dev, fetch_tree):
    """Config 4 as the bench runs it (specialised fp32, 65,536 targets, automatic schedule = the
    two-phase one: attempt 0 of every target, then the remaining attempts of the unsolved ones side
    by side): bit-identical to the same targets solved in slices of 2,048 (one phase, 4 lanes per
    target; index_base keeps each target's restart draws), and to itself over 70 back-to-back
    launches (the scratch list sets cycle)."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    N = 1 << 16
    dt = torch.float32
    Qr = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, seed=4242,
                                dtype=dt, device=dev)
    T = m.plan(arm, out_links=[gl], dtype=dt).run(Qr)[0][0].contiguous()
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt).specialize(kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
    kw = dict(max_iters=64, restarts=3, seed=0)
    ref = plan.ik_dls(T, torch.zeros((8, N), dtype=dt, device=dev), **kw)
    S = 2048
    for s in range(0, N, S):
        q, it, err = plan.ik_dls(T[:, s:s + S].contiguous(), torch.zeros((8, S), dtype=dt, device=dev),
                                 index_base=s, **kw)
        assert torch.equal(q, ref[0][:, s:s + S]) and torch.equal(it, ref[1][s:s + S]), s
        assert torch.equal(err, ref[2][:, s:s + S]), s
    outs = [plan.ik_dls(T, torch.zeros((8, N), dtype=dt, device=dev), **kw) for _ in range(70)]
    for k, o in enumerate(outs):
        assert torch.equal(o[0], ref[0]) and torch.equal(o[1], ref[1]) and torch.equal(o[2], ref[2]), k
    assert float((ref[1] <= 64).float().mean()) >= 0.99


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_ik_dls_acceptance(dev, fetch_tree, dtype):
    """Reachable random targets: converged solutions meet the reference test's criteria
    (|dp| <= 1e-3, |drpy| <= 1e-3, test/test_inverse_kinematics.jl:22-23), checked by the oracle's FK."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    ids = [j.id for j in arm]
    om = O.OracleMech(fetch_tree)
    N = 4096
    tgt = _targets(om, ids, gl.id, N, 9)
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype)
    Q = torch.zeros((8, N), dtype=dtype, device=dev)
    # axis-angle tolerance 2e-4: the reference's rpy criterion (1e-3) amplifies rotation
    # errors by up to 1/cos(pitch); it is checked below where |cos(pitch)| > 0.2 (factor <= 5)
    # the bench's solver settings (config 4: 64 iterations incl. 3 seeded restarts)
    Q, it, err = plan.ik_dls(torch.tensor(tgt, dtype=dtype, device=dev).contiguous(), Q, max_iters=64,
                             restarts=3, seed=0, tol_rot=2e-4)
    it = it.cpu().numpy()
    conv = it <= 64  # kinhip.h: max_iters + 1 <=> no attempt converged
    assert conv.mean() >= 0.99, conv.mean()
    q = Q.double().cpu().numpy()
    got = om.fk_batch(q, ids, [gl.id])[0]
    dp = np.linalg.norm(got[9:] - tgt[9:], axis=0)
    assert np.all(dp[conv] < 1e-3)
    n_rpy = 0
    for k in np.nonzero(conv)[0]:  # every converged target
        Ta, Tt = np.eye(4), np.eye(4)
        Ta[:3, :4] = got[:, k].reshape(4, 3).T
        Tt[:3, :4] = tgt[:, k].reshape(4, 3).T
        if abs(np.cos(O.rpy(Tt)[1])) > 0.2:
            d = O.rpy(Ta) - O.rpy(Tt)
            d = (d + np.pi) % (2 * np.pi) - np.pi
            assert np.all(np.abs(d) < 1e-3), (k, d)
            n_rpy += 1
    assert n_rpy > 0.9 * conv.sum()
    lo = np.array([j.lower_limit for j in arm])
    hi = np.array([j.upper_limit for j in arm])
    tol = 1e-6 if dtype == torch.float32 else 0
    assert np.all(q >= lo[:, None] - tol) and np.all(q <= hi[:, None] + tol)


def test_ik_reference_target(dev):
    """test/test_inverse_kinematics.jl:1-25: Fetch gripper to (0.3, -0.4, 1.2), identity rotation."""
    for with_base in (False, True):
        m, arm = _fetch(with_base)
        gl = m.find_link("gripper_link")
        T = np.eye(4)
        T[:3, 3] = [0.3, -0.4, 1.2]
        q, status = kinhip.inverse_kinematics_(m, gl, arm, T, with_rot=True, max_iters=200)
        assert status == ":FTOL_REACHED"
        Tn = kinhip.get_transform(m, gl)
        np.testing.assert_allclose(Tn[:3, 3], T[:3, 3], atol=1e-3)
        np.testing.assert_allclose(kinhip.rpy(Tn), kinhip.rpy(T), atol=1e-3)


@pytest.mark.parametrize("spec", [False, True])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_ik_trace_equals_separate_launches(dev, fetch_tree, spec, dtype):
    """kin_ik_dls_batch_trace (the ftol_abs rule's one launch): row k of the trace is
    bit for bit the err of a separate launch of k steps from the same seeds, for every k (restarts = 0: the
    attempt length depends on max_iters); the final angles and iteration counts equal an ordinary launch's."""
    m, arm = _fetch(False)
    gl = m.find_link("gripper_link")
    om = O.OracleMech(fetch_tree)
    N = 300
    tgt = _targets(om, [j.id for j in arm], gl.id, N, 45)
    T = torch.tensor(tgt, dtype=dtype, device=dev).contiguous()
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype)
    if spec:
        plan.specialize(kinhip.KIN_SPEC_IK)
    Q0 = torch.zeros((8, N), dtype=dtype, device=dev)
    kw = dict(lam=1e-2, tol_pos=0.0, tol_rot=0.0, max_step=0.5, with_rot=2, restarts=0, seed=3)
    M = 12
    Qt, itt, tr = plan.ik_dls_trace(T, Q0, max_iters=M, **kw)
    for k in range(M + 1):
        Q, it, err = plan.ik_dls(T, torch.empty_like(Q0), Q0=Q0, max_iters=k, lanes=1, **kw)
        assert torch.equal(tr[k], err), k
    assert torch.equal(Qt, Q) and torch.equal(itt, it)


# ------------------------------------------------------- plan specialisation ---
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("with_base", [False, True])
def test_specialized_ik_equals_generic(dev, fetch_tree, dtype, with_base):
    """KIN_SPEC_IK: specialised k_ik_dls == generic for every lane count, with_rot 0/1, the work-queue
    schedule and a base; and the specialised Nakamura kernel == generic."""
    m, arm = _fetch(with_base)
    gl = m.find_link("gripper_link")
    om = O.OracleMech(fetch_tree)
    N = 1500
    tgt = _targets(om, [j.id for j in arm], gl.id, N, 44)
    T = torch.tensor(tgt, dtype=dtype, device=dev).contiguous()
    gen = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype)
    spe = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dtype).specialize(kinhip.KIN_SPEC_IK)
    assert spe.specialized == kinhip.KIN_SPEC_IK
    nq = 8 + (3 if with_base else 0)
    for with_rot in (1, 0, 2):
        for lanes in (1, 2, 4, 8):
            kw = dict(max_iters=23, restarts=3, seed=9, lam=1e-2, max_step=0.5, lanes=lanes, with_rot=with_rot)
            a = gen.ik_dls(T, torch.zeros((nq, N), dtype=dtype, device=dev), **kw)
            b = spe.ik_dls(T, torch.zeros((nq, N), dtype=dtype, device=dev), **kw)
            # bit for bit in both precisions: the IK sources contract only inside one
            # expression (#pragma clang fp contract(on)) in both compilations, the fp32 solve runs in fp64
            assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), (with_rot, lanes)
            assert torch.equal(a[2], b[2]), (with_rot, lanes)
    if not with_base:
        gn = m.plan(arm, jac_link=gl, jac_joints=arm, with_rot=False, dtype=dtype)
        sn = m.plan(arm, jac_link=gl, jac_joints=arm, with_rot=False, dtype=dtype).specialize(
            kinhip.KIN_SPEC_NAKAMURA)
        pts = T[9:12].contiguous()
        q0 = _rand_q(N, 8, 2, dtype, dev, -0.5, 0.5)
        a = gn.point_ik_nakamura(pts, q0.clone())
        b = sn.point_ik_nakamura(pts, q0.clone())
        # 50 fixed iterations amplify last-bit differences of the two compilations: compare at the
        # fp64 parity tolerance used against the oracle (test_nakamura_vs_oracle), fp32 by residual
        if dtype == torch.float64:
            torch.testing.assert_close(a, b, atol=1e-7, rtol=0)
        else:
            pa = gen.run(a)[0][0][9:12]
            pb = gen.run(b)[0][0][9:12]
            ra, rb = (pa - pts).norm(dim=0).median(), (pb - pts).norm(dim=0).median()
            assert float(rb) < 2 * float(ra) + 1e-5


def test_specialize_errors(dev):
    """Kernel kinds that do not apply to a plan are refused (the plan keeps its generic kernels)."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    p = m.plan(arm, out_links=[gl], dtype=torch.float32)  # no Jacobian: no IK
    with pytest.raises(kinhip.KinError):
        p.specialize(kinhip.KIN_SPEC_IK)
    with pytest.raises(kinhip.KinError):
        p.specialize(kinhip.KIN_SPEC_COLL)
    assert p.specialized == 0
    assert p.specialize().specialized == kinhip.KIN_SPEC_FK


def test_launch_chunk_boundary(dev, fetch_tree):
    """Batches beyond one launch chunk (2^27 configurations: lane byte offsets stay 32-bit): the
    configurations on both sides of the chunk seam and at the tail are correct in the plain layout
    (generic kernel) and the tiled layout (specialised kernel).  FK only, fp32, ~11 GB per layout."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    N = (1 << 27) + 3000
    lo, hi = [j.lower_limit for j in arm], [j.upper_limit for j in arm]
    Q = kinhip.uniform_configs(lo, hi, N, dtype=torch.float32, device=dev)
    idx = torch.cat([torch.arange(0, 64), torch.arange((1 << 27) - 300, (1 << 27) + 300),
                     torch.arange(N - 64, N)]).to(dev)
    om = O.OracleMech(fetch_tree)
    ref = om.fk_batch(Q[:, idx].double().cpu().numpy(), [j.id for j in arm], [gl.id])
    plan = m.plan(arm, out_links=[gl], dtype=torch.float32)
    P = plan.run(Q)[0]
    np.testing.assert_allclose(P[:, :, idx].double().cpu().numpy(), ref, atol=2e-5)
    del P
    tile = 8192
    Qt = kinhip.tiled(Q, tile)
    del Q
    torch.cuda.empty_cache()
    sp = m.plan(arm, out_links=[gl], dtype=torch.float32, specialize=kinhip.KIN_SPEC_FK)
    Pt = sp.run_tiled(Qt, N)[0]
    sel = Pt[idx // tile, :, :, idx % tile]  # (len(idx), 1, 12)
    np.testing.assert_allclose(sel.permute(1, 2, 0).double().cpu().numpy(), ref, atol=2e-5)


def test_ik_launch_chunk_boundary(dev):
    """IK batches beyond one IK launch chunk (2^24 targets), specialised kernel: targets on both sides
    of the seam and at the tail converge, and their solutions reproduce the target (exact FK)."""
    m, arm = _fetch()
    gl = m.find_link("gripper_link")
    N = (1 << 24) + 1000
    lo, hi = [j.lower_limit for j in arm], [j.upper_limit for j in arm]
    Qt = kinhip.uniform_configs(lo, hi, N, seed=31, dtype=torch.float32, device=dev)
    fk = m.plan(arm, out_links=[gl], dtype=torch.float32)
    tgt = fk.run(Qt)[0][0].contiguous()
    del Qt
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32, specialize=True)
    Q, it, err = plan.ik_dls(tgt, torch.zeros((8, N), dtype=torch.float32, device=dev), max_iters=64, restarts=3)
    idx = torch.cat([torch.arange(0, 256), torch.arange((1 << 24) - 512, (1 << 24) + 512),
                     torch.arange(N - 256, N)]).to(dev)
    ok = it[idx] <= 64
    assert float(ok.float().mean()) > 0.98
    assert float((it <= 64).float().mean()) > 0.99
    P = fk.run(Q[:, idx].contiguous())[0][0]
    dp = (P[9:12] - tgt[9:12, idx]).norm(dim=0)
    assert float(dp[ok].max()) < 2e-3
