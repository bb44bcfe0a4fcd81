"""CPU oracle bindings (TEST INFRASTRUCTURE -- never imported by the product).

Only ``tests/``, ``bench.py``'s ``cpu_baseline`` leg and
``__graft_entry__.smoke()`` import this module, and only as the checker.

Two independent pieces live here:

* :func:`parse_urdf_tree` -- a Python ``xml.etree`` restatement of the URDF
  semantics Kinematics.jl gets from skrobot's vendored urdfpy
  (src/load_urdf.jl:20-80): link / joint ids in XML document order
  (1-based), ``origin`` = translation(xyz) * Rz(yaw) Ry(pitch) Rx(roll),
  ``axis`` default ``1 0 0`` normalised, joint-type map revolute /
  continuous (limits +-Inf) / prismatic / fixed, anything else raises.
  It is deliberately separate from the product's C++ URDF parser so that the
  two can be checked against each other.
* :class:`OracleMech` -- ctypes wrapper of ``oracle/_build/libkinoracle.so``,
  the C restatement of src/algorithm.jl / src/mechanism.jl /
  src/transform.jl (see kin_oracle.h for line citations).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libkinoracle.so")

FIXED, REVOLUTE, PRISMATIC = 0, 1, 2


# --------------------------------------------------------------------------
# URDF (urdfpy semantics, restated)
# --------------------------------------------------------------------------
def rpy_to_matrix(rpy):
    """urdfpy ``rpy_to_matrix``: R = Rz(y) @ Ry(p) @ Rx(r) (third-party, restated)."""
    r, p, y = (float(v) for v in rpy)
    c3, c2, c1 = math.cos(r), math.cos(p), math.cos(y)
    s3, s2, s1 = math.sin(r), math.sin(p), math.sin(y)
    return np.array([
        [c1 * c2, (c1 * s2 * s3) - (c3 * s1), (s1 * s3) + (c1 * c3 * s2)],
        [c2 * s1, (c1 * c3) + (s1 * s2 * s3), (c3 * s1 * s2) - (c1 * s3)],
        [-s2, c2 * s3, c2 * c3],
    ], dtype=np.float64)


def _origin(elem):
    T = np.eye(4)
    if elem is None:
        return T
    xyz = [float(v) for v in elem.get("xyz", "0 0 0").split()]
    rpy = [float(v) for v in elem.get("rpy", "0 0 0").split()]
    T[:3, :3] = rpy_to_matrix(rpy)
    T[:3, 3] = xyz
    return T


@dataclass
class UrdfTree:
    name: str
    link_names: list
    joint_names: list
    joint_type: np.ndarray      # int32 [J]
    joint_plink: np.ndarray     # int32 [J] 1-based
    joint_clink: np.ndarray     # int32 [J] 1-based
    joint_pose: np.ndarray      # float64 [J, 4, 4] (row-major numpy view of the 4x4)
    joint_axis: np.ndarray      # float64 [J, 3]
    joint_lower: np.ndarray
    joint_upper: np.ndarray
    link_box: dict = field(default_factory=dict)  # link id -> (extents[3], origin 4x4)

    def link_id(self, name):
        return self.link_names.index(name) + 1

    def joint_id(self, name):
        return self.joint_names.index(name) + 1


def parse_urdf_tree(path_or_text: str) -> UrdfTree:
    if os.path.exists(path_or_text):
        root = ET.parse(path_or_text).getroot()
    else:
        root = ET.fromstring(path_or_text)
    links = root.findall("link")
    joints = root.findall("joint")
    lnames = [l.get("name") for l in links]
    lid = {n: i + 1 for i, n in enumerate(lnames)}
    J = len(joints)
    jt = np.zeros(J, np.int32)
    jp = np.zeros(J, np.int32)
    jc = np.zeros(J, np.int32)
    pose = np.zeros((J, 4, 4))
    axis = np.zeros((J, 3))
    lo = np.full(J, -np.inf)
    hi = np.full(J, np.inf)
    for k, j in enumerate(joints):
        t = j.get("type")
        jp[k] = lid[j.find("parent").get("link")]
        jc[k] = lid[j.find("child").get("link")]
        pose[k] = _origin(j.find("origin"))
        ax = j.find("axis")
        a = np.array([1.0, 0.0, 0.0]) if ax is None else np.array([float(v) for v in ax.get("xyz").split()])
        n = np.linalg.norm(a)
        axis[k] = a / n if n > 0 else a
        lim = j.find("limit")
        if t == "revolute":
            jt[k] = REVOLUTE
            lo[k], hi[k] = float(lim.get("lower", 0)), float(lim.get("upper", 0))
        elif t == "continuous":
            jt[k] = REVOLUTE
        elif t == "prismatic":
            jt[k] = PRISMATIC
            lo[k], hi[k] = float(lim.get("lower", 0)), float(lim.get("upper", 0))
        elif t == "fixed":
            jt[k] = FIXED
        else:  # src/load_urdf.jl:62 throw(Exception)
            raise ValueError(f"unsupported joint type {t!r}")
    boxes = {}
    for i, l in enumerate(links):
        col = l.find("collision")
        if col is None:
            continue
        box = col.find("geometry/box")
        if box is None:
            continue
        ext = np.array([float(v) for v in box.get("size").split()])
        boxes[i + 1] = (ext, _origin(col.find("origin")))
    return UrdfTree(root.get("name"), lnames, [j.get("name") for j in joints], jt, jp, jc,
                    pose, axis, lo, hi, boxes)


# --------------------------------------------------------------------------
# C oracle
# --------------------------------------------------------------------------
class _Desc(C.Structure):
    _fields_ = [("n_links", C.c_int32), ("n_joints", C.c_int32),
                ("joint_type", C.c_void_p), ("joint_plink", C.c_void_p), ("joint_clink", C.c_void_p),
                ("joint_pose", C.c_void_p), ("joint_axis", C.c_void_p),
                ("joint_lower", C.c_void_p), ("joint_upper", C.c_void_p),
                ("with_base", C.c_int32)]


class _IkParams(C.Structure):
    _fields_ = [("max_iters", C.c_int32), ("lam", C.c_double), ("tol_pos", C.c_double),
                ("tol_rot", C.c_double), ("max_step", C.c_double), ("with_rot", C.c_int32),
                ("restarts", C.c_int32), ("seed", C.c_uint64), ("damp_err", C.c_double)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P, I32, I64, D = C.c_void_p, C.c_int32, C.c_int64, C.c_double
        L.or_mech_create.restype = P
        L.or_mech_create.argtypes = [P]
        L.or_mech_destroy.argtypes = [P]
        L.or_n_links.restype = I32
        L.or_n_links.argtypes = [P]
        L.or_set_joint_angles.argtypes = [P, I32, P, P]
        L.or_get_joint_angles.argtypes = [P, I32, P, P]
        L.or_get_transform.argtypes = [P, I32, P]
        L.or_get_jacobian.restype = C.c_int
        L.or_get_jacobian.argtypes = [P, I32, I32, P, I32, I32, P]
        L.or_is_relevant.restype = I32
        L.or_is_relevant.argtypes = [P, I32, I32]
        L.or_add_new_link.restype = I32
        L.or_add_new_link.argtypes = [P, I32, P]
        L.or_rpy.argtypes = [P, P]
        L.or_point_ik_nakamura.argtypes = [P, I32, I32, P, P, P]
        L.or_ik_objective.restype = D
        L.or_ik_objective.argtypes = [P, I32, I32, P, P, I32, P, P]
        L.or_fk_batch.argtypes = [P, I64, P, I64, I32, P, I32, P, P, I64, I32]
        L.or_fk_jac_batch.argtypes = [P, I64, P, I64, I32, P, I32, I32, P, I32, I32, I32, P, I64, P, I64, I32]
        L.or_point_ik_nakamura_batch.argtypes = [P, I64, P, I64, I32, P, I32, P, I64, I32]
        L.or_ik_dls_batch.argtypes = [P, I64, P, I64, I32, P, I32, P, I64, P, P, P, I32]
        L.or_rot_error.argtypes = [P, P, P]
        L.or_sdf_create.restype = P
        L.or_sdf_create.argtypes = [I32, P, P]
        L.or_sdf_destroy.argtypes = [P]
        L.or_box_sdf.restype = D
        L.or_box_sdf.argtypes = [P, I32, P]
        L.or_union_sdf_value.restype = D
        L.or_union_sdf_value.argtypes = [P, P, P]
        L.or_union_sdf_gradient.argtypes = [P, P, P]
        L.or_coll_batch.argtypes = [P, P, I64, P, I64, I32, P, I32, P, P, D, P, I64, P, I64, I32]
        L.or_ik_coll_batch.argtypes = [P, P, I64, P, I64, I32, P, I32, P, I64, P, P, I32, P, P, P, P, P, P, I32]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _i32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.int32))


def _f64(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64))


def tf_colmajor(T):
    """numpy 4x4 -> 16 doubles in Julia (column-major) order."""
    return _f64(np.asarray(T, dtype=np.float64).T.reshape(16))


class OracleMech:
    """Reference-faithful CPU Mechanism (one configuration at a time + batched drivers)."""

    def __init__(self, tree: UrdfTree, with_base=False):
        self.tree = tree
        self.with_base = bool(with_base)
        J = len(tree.joint_names)
        self._keep = [_i32(tree.joint_type), _i32(tree.joint_plink), _i32(tree.joint_clink),
                      _f64(np.transpose(tree.joint_pose, (0, 2, 1)).reshape(J, 16)),
                      _f64(tree.joint_axis), _f64(tree.joint_lower), _f64(tree.joint_upper)]
        d = _Desc(len(tree.link_names), J, *[_p(a).value for a in self._keep], int(self.with_base))
        self._h = lib().or_mech_create(C.byref(d))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.or_mech_destroy(self._h)
            self._h = None

    # ids --------------------------------------------------------------
    def link_id(self, name):
        return self.tree.link_id(name)

    def joint_id(self, name):
        return self.tree.joint_id(name)

    @property
    def n_links(self):
        return lib().or_n_links(self._h)

    # single-config reference API -----------------------------------------
    def set_joint_angles(self, joint_ids, angles):
        ids = _i32(joint_ids)
        a = _f64(angles)
        assert a.size == ids.size + (3 if self.with_base else 0)
        lib().or_set_joint_angles(self._h, ids.size, _p(ids), _p(a))

    def get_joint_angles(self, joint_ids):
        ids = _i32(joint_ids)
        out = np.zeros(ids.size + (3 if self.with_base else 0))
        lib().or_get_joint_angles(self._h, ids.size, _p(ids), _p(out))
        return out

    def get_transform(self, link_id):
        out = np.zeros(16)
        lib().or_get_transform(self._h, int(link_id), _p(out))
        return out.reshape(4, 4).T.copy()

    def get_jacobian(self, link_id, joint_ids, with_rot=True, rpy_jac=False, mat=None):
        ids = _i32(joint_ids)
        rows = 6 if with_rot else 3
        cols = ids.size + (3 if self.with_base else 0)
        J = np.zeros((cols, rows)) if mat is None else np.ascontiguousarray(np.asarray(mat, np.float64).T)
        rc = lib().or_get_jacobian(self._h, int(link_id), ids.size, _p(ids), int(with_rot), int(rpy_jac), _p(J))
        if rc != 0:
            raise ValueError("MethodError: joint_jacobian! has no method for a fixed joint")
        return J.T.copy()

    def is_relevant(self, joint_id, link_id):
        return bool(lib().or_is_relevant(self._h, int(joint_id), int(link_id)))

    def add_new_link(self, parent_link_id, pose4x4):
        return lib().or_add_new_link(self._h, int(parent_link_id), _p(tf_colmajor(pose4x4)))

    def point_ik_nakamura(self, link_id, joint_ids, point):
        ids = _i32(joint_ids)
        out = np.zeros(ids.size + 3)
        lib().or_point_ik_nakamura(self._h, int(link_id), ids.size, _p(ids), _p(_f64(point)), _p(out))
        return out[:ids.size]

    def ik_objective(self, link_id, joint_ids, target4x4, angles, with_rot=True):
        ids = _i32(joint_ids)
        g = np.zeros(ids.size + (3 if self.with_base else 0))
        f = lib().or_ik_objective(self._h, int(link_id), ids.size, _p(ids), _p(tf_colmajor(target4x4)),
                                  int(with_rot), _p(_f64(angles)), _p(g))
        return f, g

    # batched drivers ------------------------------------------------------
    def fk_batch(self, q, q_joint_ids, out_link_ids, n_threads=0):
        """q: [ncol, N] float64 -> poses [n_out, 12, N]"""
        q = _f64(q)
        ids, outs = _i32(q_joint_ids), _i32(out_link_ids)
        N = q.shape[1]
        poses = np.zeros((outs.size, 12, N))
        lib().or_fk_batch(self._h, N, _p(q), N, ids.size, _p(ids), outs.size, _p(outs), _p(poses), N, n_threads)
        return poses

    def fk_jac_batch(self, q, q_joint_ids, link_id, jac_joint_ids, with_rot=True, rpy_jac=False,
                     zero_fill=True, jac_init=None, n_threads=0):
        """-> pose [12, N], jac [ncol, rows, N]"""
        q = _f64(q)
        ids, jids = _i32(q_joint_ids), _i32(jac_joint_ids)
        N = q.shape[1]
        rows = 6 if with_rot else 3
        ncol = jids.size + (3 if self.with_base else 0)
        pose = np.zeros((12, N))
        jac = np.zeros((ncol, rows, N)) if jac_init is None else _f64(jac_init).copy()
        lib().or_fk_jac_batch(self._h, N, _p(q), N, ids.size, _p(ids), int(link_id), jids.size, _p(jids),
                              int(with_rot), int(rpy_jac), int(zero_fill), _p(pose), N, _p(jac), N, n_threads)
        return pose, jac

    def point_ik_nakamura_batch(self, q0, q_joint_ids, link_id, points, n_threads=0):
        q = _f64(q0).copy()
        ids = _i32(q_joint_ids)
        pts = _f64(points)
        N = q.shape[1]
        lib().or_point_ik_nakamura_batch(self._h, N, _p(q), N, ids.size, _p(ids), int(link_id), _p(pts),
                                         pts.shape[1], n_threads)
        return q

    def ik_dls_batch(self, q0, q_joint_ids, link_id, target, max_iters=64, lam=1e-2, tol_pos=1e-3,
                     tol_rot=1e-3, max_step=0.5, with_rot=True, restarts=0, seed=0, n_threads=0, damp_err=0.0):
        q = _f64(q0).copy()
        ids = _i32(q_joint_ids)
        tgt = _f64(target)
        N = q.shape[1]
        it = np.zeros(N, np.int32)
        err = np.zeros((2, N))
        prm = _IkParams(max_iters, lam, tol_pos, tol_rot, max_step, int(with_rot), int(restarts), int(seed),
                        float(damp_err))
        lib().or_ik_dls_batch(self._h, N, _p(q), N, ids.size, _p(ids), int(link_id), _p(tgt), tgt.shape[1],
                              C.byref(prm), _p(it), _p(err), n_threads)
        return q, it, err


def ik_coll_batch(mech: "OracleMech", sdf: "OracleUnionSDF", q0, q_joint_ids, link_id, target, sphere_links, radii,
                  margin=0.02, band=0.01, weight=1.0, feas=1e-6, max_iters=64, lam=1e-2, tol_pos=1e-3, tol_rot=1e-3,
                  max_step=0.5, with_rot=2, restarts=0, seed=0, n_threads=0, sdfs=None, sphere_parents=None,
                  q_alt=None):
    """Restatement of kin_ik_coll_batch (stage 2 of the bistage collision-aware IK) -> (q, iters, err [3, N]).
    `q_alt` (the layout of q0): kin_ik_coll_batch_alt's restart origin (attempt 1's joints, every restart's base).
    `sdfs`: one OracleUnionSDF per target (a scene mechanism's boxes at each target's scene state) instead of
    `sdf`.  `sphere_parents`: the tree links the sphere links hang off (add_new_link parents); with it the
    sphere rows are added in the kernel's order (ikc_sphere_order) -- the same sums in the same order."""
    q = _f64(q0).copy()
    ids = _i32(q_joint_ids)
    tgt = _f64(target)
    sph = _i32(sphere_links)
    r = _f64(radii)
    if sphere_parents is not None and sph.size:
        order = ikc_sphere_order(mech.tree, ids, int(link_id), _i32(sphere_parents))
        sph, r = _i32(sph[order]), _f64(r[order])
    N = q.shape[1]
    it = np.zeros(N, np.int32)
    err = np.zeros((3, N))
    prm = _IkParams(max_iters, lam, tol_pos, tol_rot, max_step, int(with_rot), int(restarts), int(seed))
    cp = _f64([margin, band, weight, feas])
    qa = None if q_alt is None else _f64(q_alt)
    assert qa is None or qa.shape == q.shape
    harr = None
    if sdfs is not None:
        assert len(sdfs) == N
        harr = (C.c_void_p * N)(*[s._h for s in sdfs])
    lib().or_ik_coll_batch(mech._h, (sdf or sdfs[0])._h, N, _p(q), N, ids.size, _p(ids), int(link_id), _p(tgt),
                           tgt.shape[1], C.byref(prm), _p(cp), sph.size, _p(sph) if sph.size else None,
                           _p(r) if sph.size else None, C.cast(harr, C.c_void_p) if harr is not None else None,
                           _p(qa) if qa is not None else None, _p(it), _p(err), n_threads)
    return q, it, err


def ikc_sphere_order(tree: UrdfTree, q_joint_ids, link_id, sphere_links):
    """The order in which kin_ik_coll_batch adds the sphere rows (kinhip_host.cpp stage_ikc_tree): spheres on
    the root frame first, then by the depth-first position (children in joint order) of the moving joint
    whose frame carries them, the caller's order inside a carrier."""
    J = len(tree.joint_names)
    cols = {}
    for c, j in enumerate(q_joint_ids):
        cols[int(j)] = c  # a repeated joint keeps its last column
    moving = {j for j in cols if tree.joint_type[j - 1] != FIXED}
    pjoint = {int(tree.joint_clink[j - 1]): j for j in range(1, J + 1)}
    needed = set()

    def mark(l):
        while l is not None and l not in needed:
            needed.add(l)
            pj = pjoint.get(l)
            l = int(tree.joint_plink[pj - 1]) if pj else None

    mark(int(link_id))
    for l in sphere_links:
        mark(int(l))
    children = {}
    for j in range(1, J + 1):
        children.setdefault(int(tree.joint_plink[j - 1]), []).append(j)
    carrier = {}
    count = [0]

    def visit(x, car):
        carrier[x] = car
        for j in children.get(x, []):
            c = int(tree.joint_clink[j - 1])
            if c not in needed:
                continue
            if j in moving:
                s = count[0]
                count[0] += 1
                visit(c, s)
            else:
                visit(c, car)

    for l in range(1, len(tree.link_names) + 1):
        if l in needed and l not in pjoint:
            visit(l, -1)
    return sorted(range(len(sphere_links)), key=lambda k: (carrier[int(sphere_links[k])], k))


def rot_error(T_target, T_now):
    """The DLS IK's rotation error: log(R* R^T) as a world rotation vector (or_rot_error)."""
    a, b = tf_colmajor(T_target), tf_colmajor(T_now)
    w = np.zeros(3)
    lib().or_rot_error(_p(a), _p(b), _p(w))
    return w


def rpy(T):
    out = np.zeros(3)
    lib().or_rpy(_p(tf_colmajor(T)), _p(out))
    return out


class OracleUnionSDF:
    """UnionSDF of BoxSDFs (src/sdf.jl:48-114): boxes given by world pose (4x4) and full widths."""

    def __init__(self, poses, widths):
        poses = np.asarray(poses, np.float64).reshape(-1, 4, 4)
        self.n = poses.shape[0]
        P = _f64(np.transpose(poses, (0, 2, 1)).reshape(-1))
        W = _f64(np.asarray(widths, np.float64).reshape(-1))
        self._h = lib().or_sdf_create(self.n, _p(P), _p(W))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.or_sdf_destroy(self._h)
            self._h = None

    def box(self, k, p):
        return lib().or_box_sdf(self._h, int(k), _p(_f64(p)))

    def __call__(self, p):
        return lib().or_union_sdf_value(self._h, _p(_f64(p)), None)

    def gradient(self, p):
        g = np.zeros(3)
        lib().or_union_sdf_gradient(self._h, _p(_f64(p)), _p(g))
        return g


def coll_batch(mech: "OracleMech", sdf: OracleUnionSDF, q, q_joint_ids, sphere_links, radii, truncation=np.inf,
               with_grad=True, n_threads=0):
    """-> dists [n_sph, N], grads [n_sph, n_dof, N] (compute_coll_dists_and_grads!, src/collision.jl:67-94)."""
    q = _f64(q)
    ids = _i32(q_joint_ids)
    sph = _i32(sphere_links)
    r = _f64(radii)
    N = q.shape[1]
    ndof = ids.size + (3 if mech.with_base else 0)
    d = np.zeros((sph.size, N))
    g = np.zeros((sph.size, ndof, N)) if with_grad else None
    lib().or_coll_batch(mech._h, sdf._h, N, _p(q), N, ids.size, _p(ids), sph.size, _p(sph), _p(r),
                        float(truncation), _p(d), N, _p(g) if with_grad else None, N, n_threads)
    return d, g


def fridge_boxes(tree: UrdfTree, door_angle=2.0, base=(1.2, 0.0, 0.0)):
    """UnionSDF(fridge) of test/test_inverse_kinematics.jl:52-70: one BoxSDF per URDF link with a box
    collision, attached at the collision origin (src/sdf.jl:82-97), world poses with the fridge's
    planar base and door joint set."""
    m = OracleMech(tree, with_base=True)
    door = tree.joint_id("door_joint")
    m.set_joint_angles([door], [door_angle, *base])
    poses, widths = [], []
    for lid, (ext, org) in sorted(tree.link_box.items()):
        poses.append(m.get_transform(lid) @ org)
        widths.append(ext)
    return np.array(poses), np.array(widths)


# ---------------------------------------------------------------------------
# Planning constraints (src/planning.jl), restated on top of the functions above
# ---------------------------------------------------------------------------
def ineq_const(mech: "OracleMech", sdf: OracleUnionSDF, xi, q_joint_ids, sphere_links, radii, n_wp, margin):
    """IneqConst(xi, val_vec, jac_mat), src/planning.jl:55-68: per waypoint i the spheres'
    dists (truncated at margin + 0.05) minus margin, and the block-diagonal jac_mat
    [n_dof*n_wp, n_coll*n_wp] of their gradients."""
    xi = np.asarray(xi, np.float64)
    n_dof = xi.size // n_wp
    Q = xi.reshape(n_wp, n_dof).T  # reshape(xi, (n_dof, n_wp)), column-major
    d, g = coll_batch(mech, sdf, Q, q_joint_ids, sphere_links, radii, truncation=margin + 0.05)
    n_coll = d.shape[0]
    val = np.zeros(n_coll * n_wp)
    jac = np.zeros((n_dof * n_wp, n_coll * n_wp))
    for i in range(n_wp):
        jac[n_dof * i:n_dof * (i + 1), n_coll * i:n_coll * (i + 1)] = g[:, :, i].T
        val[n_coll * i:n_coll * (i + 1)] = d[:, i] - margin
    return val, jac


def pose_const(mech: "OracleMech", q, q_joint_ids, link_id, target4x4, with_rot):
    """PoseConstraint for one link, src/planning.jl:114-138: [p - p*; rpy - rpy*] and the
    rpy Jacobian (get_jacobian!(..., rpy_jac=true)) as [dim, n_dof]."""
    q = np.asarray(q, np.float64).reshape(-1, 1)
    ids = list(q_joint_ids)
    pose, J = mech.fk_jac_batch(q, ids, link_id, ids, with_rot=with_rot, rpy_jac=True)
    cur = np.eye(4)
    cur[:3, :] = pose[:, 0].reshape(4, 3).T
    T = np.asarray(target4x4, np.float64)
    diff = cur[:3, 3] - T[:3, 3]
    if with_rot:
        diff = np.concatenate([diff, rpy(cur) - rpy(T)])
    return diff, J[:, :, 0].T  # J: [ncol, rows, 1] -> [rows, ncol]
