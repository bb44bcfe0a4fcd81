"""The headline path at the north star's tolerance: Fetch FK + 6x8 J in fp32 through the bench's exact
kernel (plan-specialised k_fk, tiled SoA, tile 8192) within 1e-6 absolute of the reference algorithm.

The reference computes in fp64 (test/test_kinematics.jl:10-41 pins it at 1e-6 on ground_truth.json).
An fp32 engine sees its angles rounded to fp32 first (a caller's Float32 array), so the comparison is
against the oracle (pinned to ground_truth.json at 4.4e-16) evaluated at those same fp32 angles: the
residual is the engine's own fp32 arithmetic.  ground_truth.json itself is also run through the fp32
headline path, where the angle rounding is included in the residual.
"""
import json

import numpy as np
import pytest
import torch

import oracle as O
from conftest import ARM, golden

import kinhip

pytestmark = pytest.mark.gpu

TOL32 = 1e-6  # BASELINE north star: link poses and Jacobian entries within 1e-6 absolute


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda", 0)


def _headline_plan(m, arm, gl):
    return m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32).specialize(kinhip.KIN_SPEC_FK)


@pytest.mark.parametrize("start", [0, 7 * (1 << 20)])
def test_headline_fp32_full_batch_vs_oracle(dev, start):
    """The bench's dataset (2^20 counter-hashed within-limit configurations; a second, later slice as a
    rank > 0 would draw it), the bench's kernel and layout, all 2^20 x 60 outputs vs the fp64 oracle."""
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    gl = m.find_link("gripper_link")
    N, tile = 1 << 20, 8192
    Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, start=start,
                               dtype=torch.float32, device=dev)
    Pt, Jt = _headline_plan(m, arm, gl).run_tiled(kinhip.tiled(Q, tile), N)
    pose = kinhip.untiled(Pt, N)[0].double().cpu().numpy()
    jac = kinhip.untiled(Jt, N).double().cpu().numpy()
    om = O.OracleMech(O.parse_urdf_tree(golden("fetch.urdf")))
    ids = [j.id for j in arm]
    ps, js = om.fk_jac_batch(Q.double().cpu().numpy(), ids, gl.id, ids, True, False)
    ep, ej = float(np.abs(pose - ps).max()), float(np.abs(jac - js).max())
    print(f"fp32 headline vs oracle at 2^20: max|pose| {ep:.3e}, max|J| {ej:.3e}")
    assert ep <= TOL32 and ej <= TOL32, (ep, ej)


def test_golden_fixture_fp32_at_north_star(dev):
    """tests/golden/fetch_fk_jac_golden.npz (all 25 links, 6x8 J of gripper_link): fp32 engine vs the
    fixture's generator (the oracle, 1e-12 to the fixture) at the fp32-rounded fixture angles."""
    g = np.load(golden("fetch_fk_jac_golden.npz"))
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    gl = m.find_link("gripper_link")
    om = O.OracleMech(O.parse_urdf_tree(golden("fetch.urdf")))
    ids = [j.id for j in arm]
    q32 = torch.tensor(g["q"], dtype=torch.float32, device=dev).contiguous()
    q32d = q32.double().cpu().numpy()
    # the oracle reproduces the fixture at the fixture's own (fp64) angles
    ps64, js64 = om.fk_jac_batch(g["q"], ids, gl.id, ids, True, False)
    assert np.abs(js64 - g["jac_geo"]).max() < 1e-12 and np.abs(ps64 - g["poses"][gl.id - 1]).max() < 1e-12
    N = q32.shape[1]
    Pt, Jt = _headline_plan(m, arm, gl).run_tiled(kinhip.tiled(q32, 256), N)
    ps, js = om.fk_jac_batch(q32d, ids, gl.id, ids, True, False)
    assert np.abs(kinhip.untiled(Pt, N)[0].double().cpu().numpy() - ps).max() <= TOL32
    assert np.abs(kinhip.untiled(Jt, N).double().cpu().numpy() - js).max() <= TOL32
    allp = kinhip.get_transform_batch(m, m.links, arm, q32).double().cpu().numpy()
    ref = om.fk_batch(q32d, ids, [l.id for l in m.links])
    assert np.abs(allp - ref).max() <= TOL32


@pytest.mark.parametrize("with_base", [False, True])
def test_ground_truth_json_fp32_headline_kernel(dev, with_base):
    """test/test_kinematics.jl:10-41: ground_truth.json (PR2 fragment, 9 links) through the fp32
    specialised tiled kernel, translation and RotZYX angles within 1e-6 of the file."""
    gt = json.load(open(golden("ground_truth.json")))
    m = kinhip.parse_urdf(golden("pr2_torso_rarm.urdf"), with_base=with_base)
    joints = [m.find_joint(n) for n in gt["joint_names"]]
    links = [m.find_link(n) for n in gt["link_names"]]
    angles = list(gt["angle_vector"]) + ([0.3, 0.3, 0.3] if with_base else [])
    n = 300  # two tiles of 256, the second partial
    Q = torch.tensor(angles, dtype=torch.float32, device=dev).reshape(-1, 1).repeat(1, n).contiguous()
    sp = m.plan(joints, out_links=links, dtype=torch.float32).specialize(kinhip.KIN_SPEC_FK)
    Pt, _ = sp.run_tiled(kinhip.tiled(Q, 256), n)
    poses = kinhip.untiled(Pt, n).double().cpu().numpy()
    assert np.array_equal(poses[..., :1].repeat(n, axis=2), poses)
    th = 0.3
    Rz = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
    worst = 0.0
    for k, pg in enumerate(gt["pose_list"]):
        T = np.eye(4)
        T[:3, :4] = poses[k, :, 0].reshape(4, 3).T
        r = kinhip.rpy(T)
        ypr = np.array([r[2], r[1], r[0]])
        pg = np.asarray(pg)
        if with_base:
            et, er = np.abs(T[:3, 3] - (Rz @ pg[:3] + [0.3, 0.3, 0])), np.abs(ypr - (pg[3:] + [0.3, 0, 0]))
        else:
            et, er = np.abs(T[:3, 3] - pg[:3]), np.abs(ypr - pg[3:])
        worst = max(worst, float(et.max()), float(er.max()))
    print(f"ground_truth.json through the fp32 headline kernel: max abs error {worst:.3e}")
    assert worst <= TOL32, worst


def test_config2_bench_path_full_batch_vs_oracle(dev):
    """config 2's exact bench path -- FK of the 6 exampel.jl:11 links in fp64, the
    plan-specialised kernel on the tiled layout (tile 4096), the bench's 2^20 counter-hashed dataset --
    every one of the 2^20 x 6 x 12 outputs against the fp64 oracle at 1e-9 (the fp64 gate)."""
    from conftest import EXAMPLE_LINKS
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    links = [m.find_link(n) for n in EXAMPLE_LINKS]
    N, tile = 1 << 20, 4096
    Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], N, dtype=torch.float64,
                               device=dev)
    plan = m.plan(arm, out_links=links, dtype=torch.float64).specialize(kinhip.KIN_SPEC_FK)
    Pt, _ = plan.run_tiled(kinhip.tiled(Q, tile), N)
    got = kinhip.untiled(Pt, N).cpu().numpy()  # [6, 12, N]
    om = O.OracleMech(O.parse_urdf_tree(golden("fetch.urdf")))
    ref = om.fk_batch(Q.cpu().numpy(), [j.id for j in arm], [l.id for l in links])
    e = float(np.abs(got - ref).max())
    print(f"config 2 bench path vs oracle at 2^20: max|pose| {e:.3e}")
    assert e <= 1e-9, e
