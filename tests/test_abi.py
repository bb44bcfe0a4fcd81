"""C-ABI and host logic of libkinhip.so, no GPU compute (runs in the CPU container).

 - the library loads and exports every entry point include/kinhip.h declares
 - the native URDF parser agrees with the oracle's independent xml.etree reader
   (ids in document order, joint types, 4x4 origins, normalised axes, limits,
   box collision metadata) on fetch.urdf, fridge.urdf and the PR2 fragment
 - Mechanism host mirror: tree queries and rptable facts of test/test_mechanism.jl,
   add_new_link, KeyError / MethodError behaviour, malformed trees rejected
 - the fp32 atan2 polynomial's constants in kinhip_device.h (host evaluation)
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle as O
from conftest import ROOT, golden

import kinhip
from kinhip import _lib as K


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "kinhip.h")).read()
    return sorted(set(re.findall(r"KINHIP_API\s+[\w\s\*]+?\b(kin_\w+)\s*\(", src)))


def test_exports_every_declared_symbol():
    L = K.lib()
    decl = _header_symbols()
    assert len(decl) >= 25
    missing = [s for s in decl if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(K.EXPORTS) == decl
    assert L.kin_abi_version() == 2
    mc, mj, ms = C.c_int32(), C.c_int32(), C.c_int32()
    assert L.kin_limits(C.byref(mc), C.byref(mj), C.byref(ms)) == 0
    assert (mc.value, mj.value, ms.value) == (32, 64, 8)


@pytest.mark.parametrize("fname", ["fetch.urdf", "fridge.urdf", "pr2_torso_rarm.urdf"])
def test_urdf_parser_matches_reference_semantics(fname):
    ref = O.parse_urdf_tree(golden(fname))
    m = kinhip.parse_urdf(golden(fname))
    assert [l.name for l in m.links] == ref.link_names
    assert [j.name for j in m.joints] == ref.joint_names
    for k, j in enumerate(m.joints):
        assert K._lib is not None
        assert {"fixed": 0, "revolute": 1, "prismatic": 2}[j.jtype] == ref.joint_type[k]
        assert (j.plink_id, j.clink_id) == (ref.joint_plink[k], ref.joint_clink[k])
        np.testing.assert_allclose(j.pose, ref.joint_pose[k], atol=1e-15)
        if j.jtype != "fixed":
            np.testing.assert_allclose(j.axis, ref.joint_axis[k], atol=1e-15)
        assert j.lower_limit == ref.joint_lower[k] and j.upper_limit == ref.joint_upper[k]
    for lid, (ext, org) in ref.link_box.items():
        meta = m.links[lid - 1].geometric_meta_data
        np.testing.assert_allclose(meta.extents, ext)
        np.testing.assert_allclose(meta.origin, org, atol=1e-15)
    assert sum(l.geometric_meta_data is not None for l in m.links) == len(ref.link_box)


def test_mechanism_tree_queries():
    """test/test_mechanism.jl:1-29 through the product's host mirror."""
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    base = kinhip.find_link(m, "base_link")
    assert {l.name for l in kinhip.child_links(m, base)} == {
        "r_wheel_link", "l_wheel_link", "torso_lift_link", "estop_link", "laser_link", "torso_fixed_link"}
    assert kinhip.isroot(base) and base.pjoint_id == -1
    sh = kinhip.find_link(m, "shoulder_pan_link")
    assert kinhip.parent_joint(m, sh).name == "shoulder_pan_joint"
    assert kinhip.parent_link(m, sh).name == "torso_lift_link"
    assert [l.name for l in kinhip.child_links(m, sh)] == ["shoulder_lift_link"]
    assert [j.name for j in kinhip.child_joints(m, sh)] == ["shoulder_lift_joint"]
    for leaf in ["r_wheel_link", "l_wheel_link", "r_gripper_finger_link", "l_gripper_finger_link", "bellows_link2",
                 "estop_link", "laser_link", "torso_fixed_link", "head_camera_rgb_optical_frame",
                 "head_camera_depth_optical_frame"]:
        link = kinhip.find_link(m, leaf)
        assert kinhip.isleaf(link) and not link.cjoint_ids
    with pytest.raises(KeyError):
        kinhip.find_link(m, "no_such_link")


def test_rptable_and_add_new_link():
    """test/test_mechanism.jl:54-67: is_relevant through the C-ABI, then add_new_link."""
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    fj, fl = m.find_joint, m.find_link
    assert kinhip.is_relevant(m, fj("torso_lift_joint"), fl("torso_lift_link"))
    assert kinhip.is_relevant(m, fj("shoulder_pan_joint"), fl("wrist_roll_link"))
    assert not kinhip.is_relevant(m, fj("shoulder_pan_joint"), fl("base_link"))
    ref = O.OracleMech(O.parse_urdf_tree(golden("fetch.urdf")))
    for j in m.joints:  # the whole table against the oracle's create_rptable
        for l in m.links:
            assert kinhip.is_relevant(m, j, l) == ref.is_relevant(j.id, l.id)
    new = kinhip.Link("mylink", link_type="User")
    kinhip.add_new_link(m, new, fl("wrist_roll_link"), [0, 0, 0])
    assert new.id == 26 and m.find_link("mylink") is new
    assert m.find_joint("mylink_joint").jtype == "fixed"
    assert kinhip.is_relevant(m, fj("torso_lift_joint"), new)
    assert not kinhip.is_relevant(m, fj("head_pan_joint"), new)


def test_joint_angle_state():
    m = kinhip.parse_urdf(golden("fetch.urdf"), with_base=True)
    js = [m.find_joint(n) for n in ["torso_lift_joint", "shoulder_pan_joint"]]
    with pytest.raises(AssertionError):
        m.set_joint_angles(js, [0.1, 0.2])  # with_base needs 3 more values (mechanism.jl:224)
    m.set_joint_angles(js, [0.1, 0.2, 1.0, 2.0, 3.0])
    np.testing.assert_array_equal(m.get_joint_angles(js), [0.1, 0.2, 1.0, 2.0, 3.0])
    assert m.joint_angle(js[1]) == 0.2


def _desc(types, plink, clink, n_links):
    J = len(types)
    arrs = [np.array(types, np.int32), np.array(plink, np.int32), np.array(clink, np.int32),
            np.tile(np.eye(4).reshape(16), J).astype(np.float64), np.tile([0, 0, 1.0], J)]
    d = K.TreeDesc(n_links, J, *[a.ctypes.data for a in arrs], None, None, 0)
    return d, arrs


@pytest.mark.parametrize("types,plink,clink,nl,code", [
    ([1], [1], [3], 2, K.KIN_E_KEY),          # child id out of range
    ([7], [1], [2], 2, K.KIN_E_INVALID),      # unknown joint type
    ([1, 1], [1, 1], [2, 2], 2, K.KIN_E_INVALID),   # link with two parents
    ([1, 1], [1, 2], [2, 1], 2, K.KIN_E_INVALID),   # cycle
])
def test_model_create_rejects_malformed(types, plink, clink, nl, code):
    d, keep = _desc(types, plink, clink, nl)
    h = C.c_void_p()
    assert K.lib().kin_model_create(C.byref(d), C.byref(h)) == code
    assert K.lib().kin_last_error()


def test_urdf_errors():
    L = K.lib()
    h = C.c_void_p()
    bad = b"<robot name='x'><link name='a'/><link name='b'/><joint name='j' type='floating'>" \
          b"<parent link='a'/><child link='b'/></joint></robot>"
    assert L.kin_urdf_parse_string(bad, len(bad), C.byref(h)) == K.KIN_E_PARSE
    assert b"floating" in L.kin_last_error()
    assert L.kin_urdf_parse_string(b"<robot><link", 12, C.byref(h)) == K.KIN_E_PARSE
    assert L.kin_urdf_parse_file(b"/nonexistent.urdf", C.byref(h)) == K.KIN_E_IO
    ok = b"<?xml version='1.0'?><!-- c --><robot name='r'><link name='a'/></robot>"
    assert L.kin_urdf_parse_string(ok, len(ok), C.byref(h)) == 0
    lid = C.c_int32()
    assert L.kin_urdf_find_link(h, b"a", C.byref(lid)) == 0 and lid.value == 1
    assert L.kin_urdf_find_link(h, b"zz", C.byref(lid)) == K.KIN_E_KEY
    L.kin_urdf_destroy(h)


def test_plan_errors_before_device():
    """Plan validation (ids, MethodError) happens on the host, before any device work."""
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
    with pytest.raises(TypeError):  # relevant fixed joint: no joint_jacobian! method
        m.plan(arm, jac_link=m.find_link("gripper_link"), jac_joints=[m.find_joint("gripper_axis")])
    bogus = kinhip.Joint("bogus", 999, 1, 2, np.eye(4), "revolute", np.array([0, 0, 1.0]))
    with pytest.raises(KeyError):
        m.plan([bogus], out_links=[m.find_link("gripper_link")])


def test_synthetic_configs_are_shard_invariant():
    import torch
    lo, hi = [0.0, -1.0, -np.inf], [0.4, 1.0, np.inf]
    full = kinhip.uniform_configs(lo, hi, 1000, start=0, dtype=torch.float64)
    a = kinhip.uniform_configs(lo, hi, 400, start=0, dtype=torch.float64)
    b = kinhip.uniform_configs(lo, hi, 600, start=400, dtype=torch.float64)
    assert torch.equal(full, torch.cat([a, b], 1))
    assert float(full[0].min()) >= 0 and float(full[0].max()) <= 0.4
    assert float(full[2].min()) >= -np.pi and float(full[2].max()) <= np.pi
    assert abs(float(full[1].mean())) < 0.1


def test_reference_host_helpers():
    """Host-side mirrors of the reference exports (src/transform.jl, src/mechanism.jl)."""
    import numpy as np
    import kinhip
    import oracle as O
    from conftest import golden
    R = O.rpy_to_matrix([0.3, -0.4, 1.1])
    T = kinhip.Transform(R, [1.0, 2.0, 3.0])
    np.testing.assert_allclose(kinhip.rotation(T), R)
    np.testing.assert_allclose(kinhip.translation(T), [1, 2, 3])
    np.testing.assert_allclose(kinhip.rpy(T), O.rpy(T), atol=1e-15)
    np.testing.assert_allclose(kinhip.rpy(T), [0.3, -0.4, 1.1], atol=1e-12)
    np.testing.assert_array_equal(kinhip.Transform(), np.eye(4))
    m = kinhip.parse_urdf(golden("fetch.urdf"))
    j = m.find_joint("elbow_flex_joint")
    kinhip.set_joint_angle(m, j, -0.7)
    assert kinhip.joint_angle(m, j) == -0.7
    out = np.zeros(2)
    kinhip.get_joint_angles_(m, [m.find_joint("shoulder_pan_joint"), j], out)
    np.testing.assert_array_equal(out, [0.0, -0.7])
    c, r = kinhip.compute_swept_sphere(m.find_link("upperarm_roll_link"))
    assert len(c) == len(r) == 2 and all(x > 0 for x in r)
    assert kinhip.compute_swept_sphere(m.find_link("base_link")) == ([], [])


def test_jit_selfcheck_compiles_on_host():
    """Plan specialisation's run-time compilation (hiprtc, gfx950) of every kernel kind in both
    precisions works without a GPU: the embedded device sources compile as a hiprtc program."""
    import time
    t0 = time.perf_counter()
    rc = K.lib().kin_jit_selfcheck()
    msg = K.lib().kin_last_error()
    assert rc == K.KIN_OK, (msg or b"").decode()[:2000]
    assert time.perf_counter() - t0 < 120


def test_fp32_atan2_polynomial_constants():
    """atan2_pos_fast (kinhip_device.h, the fp32 IK's rotation-error angle): the coefficients in
    the header, evaluated in fp32 with the device's octant reduction, stay within 4e-7 of atan2
    over [0, pi] (the fit is tools/atan_fit.py)."""
    src = open(os.path.join(ROOT, "kinematics.jl_amd", "csrc", "kinhip_device.h")).read()
    body = src[src.index("float atan2_pos_fast(float s, float c)"):]
    body = body[:body.index("\n}\n")]
    cf = [float(x) for x in re.findall(r"p = (?:fmaf\(p, z, )?(-?[0-9.]+)f", body)]
    assert len(cf) == 7
    f = np.float32
    th = np.linspace(0.0, np.pi, 400001)
    for rad in (1.0, 0.25, 1e-3):
        s, c = (rad * np.sin(th)).astype(f), (rad * np.cos(th)).astype(f)
        ac = np.abs(c)
        mx, mn = np.maximum(s, ac), np.minimum(s, ac)
        a = np.where(mx > 0, mn / np.where(mx > 0, mx, f(1)), f(0)).astype(f)
        z = a * a
        p = f(cf[0])
        for k in cf[1:]:
            p = (p * z + f(k)).astype(f)
        r = (a * z * p + a).astype(f)
        r = np.where(s > ac, f(1.57079633) - r, r)
        r = np.where(c < 0, f(3.14159265) - r, r)
        ref = np.arctan2(s.astype(np.float64), c.astype(np.float64))
        assert np.abs(r.astype(np.float64) - ref).max() < 4e-7
