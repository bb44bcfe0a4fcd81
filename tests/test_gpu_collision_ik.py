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
