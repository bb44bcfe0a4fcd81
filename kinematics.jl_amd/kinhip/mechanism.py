"""Host-side mirror of Kinematics.jl's Mechanism API over libkinhip.so.

Mirrors the reference's exported names and their meaning (src/Kinematics.jl:45-73):
``parse_urdf``, ``Mechanism``, ``Link``, ``Joint``, ``find_link`` /
``find_joint`` (KeyError on unknown names), ``parent_link`` ...,
``set_joint_angles`` / ``get_joint_angles``, ``is_relevant``,
``add_new_link``, ``get_transform``, ``get_jacobian`` / ``get_jacobian_``
(Julia's ``get_jacobian!``), ``rpy``.  The single-configuration calls run the
HIP engine with a batch of one; the batched calls (``Plan``,
``get_transform_batch``, ``get_jacobian_batch``) are the hot path.

Array layout of the batched calls = Julia column-major ``Matrix{T}(N, k)``:
torch tensors of shape ``(k, N)`` (configuration index fastest); poses
``(n_links, 12, N)`` (3x4 column-major per link); Jacobians
``(n_cols, rows, N)``.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib as K

_DT = {torch.float32: K.KIN_F32, torch.float64: K.KIN_F64}


# ---------------------------------------------------------------------------
# data types (src/mechanism.jl:1-88)
# ---------------------------------------------------------------------------
@dataclass
class BoxMetaData:
    extents: np.ndarray
    origin: np.ndarray  # 4x4


@dataclass
class SphereMetaData:
    radius: float
    origin: np.ndarray


@dataclass(eq=False)
class Link:
    name: str
    id: int = -1
    pjoint_id: int = -1
    cjoint_ids: list = field(default_factory=list)
    plink_id: int = -1
    clink_ids: list = field(default_factory=list)
    geometric_meta_data: object = None
    link_type: str = "URDF"
    data: dict = field(default_factory=dict)


@dataclass(eq=False)
class Joint:
    name: str
    id: int
    plink_id: int
    clink_id: int
    pose: np.ndarray  # 4x4
    jtype: str        # "revolute" (incl. continuous), "prismatic", "fixed"
    axis: np.ndarray
    lower_limit: float = -math.inf
    upper_limit: float = math.inf


_JT = {K.KIN_JOINT_FIXED: "fixed", K.KIN_JOINT_REVOLUTE: "revolute", K.KIN_JOINT_PRISMATIC: "prismatic"}
_JT_INV = {v: k for k, v in _JT.items()}


def _i32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.int32))


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _ids(items) -> np.ndarray:
    return _i32([it.id if hasattr(it, "id") else int(it) for it in items])


class Mechanism:
    """Kinematic tree + state (src/mechanism.jl:147-181), backed by a kin_model."""

    def __init__(self, links: list, joints: list, with_base: bool = False, name: str = "basic"):
        self.name = name
        self.links = links
        self.joints = joints
        self.with_base = bool(with_base)
        self.linkid_map = {l.name: l.id for l in links}
        self.jointid_map = {j.name: j.id for j in joints}
        self.angles = np.zeros(len(joints))
        self.base_pose = np.zeros(3)
        self._angles_synced = True
        self._model = C.c_void_p()
        self._create_model()

    # -- native model ---------------------------------------------------------
    def _tree_arrays(self):
        J = len(self.joints)
        return [_i32([_JT_INV[j.jtype] for j in self.joints]), _i32([j.plink_id for j in self.joints]),
                _i32([j.clink_id for j in self.joints]),
                np.ascontiguousarray(np.array([np.asarray(j.pose, np.float64).T.reshape(16) for j in self.joints]
                                              ).reshape(J * 16) if J else np.zeros(16)),
                np.ascontiguousarray(np.array([j.axis for j in self.joints], np.float64).reshape(-1) if J else np.zeros(3)),
                np.array([j.lower_limit for j in self.joints], np.float64),
                np.array([j.upper_limit for j in self.joints], np.float64)]

    def _create_model(self):
        arrs = self._tree_arrays()
        d = K.TreeDesc(len(self.links), len(self.joints), *[_p(a).value for a in arrs], int(self.with_base))
        K.check(K.lib().kin_model_create(C.byref(d), C.byref(self._model)))

    def __del__(self):
        if getattr(self, "_model", None) and K._lib is not None:
            K._lib.kin_model_destroy(self._model)
            self._model = None

    def _sync_angles(self):
        if not self._angles_synced:
            a = np.ascontiguousarray(self.angles, np.float64)
            K.check(K.lib().kin_model_set_angles(self._model, _p(a)))
            self._angles_synced = True

    # -- tree queries (src/mechanism.jl:183-197) -----------------------------
    def find_link(self, name) -> Link:
        return self.links[self.linkid_map[name] - 1]  # KeyError like Julia's Dict

    def find_joint(self, name) -> Joint:
        return self.joints[self.jointid_map[name] - 1]

    def parent_link(self, x):
        return self.links[x.plink_id - 1]

    def child_link(self, joint: Joint) -> Link:
        return self.links[joint.clink_id - 1]

    def child_links(self, link: Link):
        return [self.links[i - 1] for i in link.clink_ids]

    def parent_joint(self, link: Link) -> Joint:
        return self.joints[link.pjoint_id - 1]

    def child_joints(self, link: Link):
        return [self.joints[i - 1] for i in link.cjoint_ids]

    def is_relevant(self, joint: Joint, link: Link) -> bool:
        out = C.c_int32()
        K.check(K.lib().kin_model_is_relevant(self._model, joint.id, link.id, C.byref(out)))
        return bool(out.value)

    # -- state (src/mechanism.jl:197-231) ------------------------------------
    def joint_angle(self, joint: Joint) -> float:
        return float(self.angles[joint.id - 1])

    def set_joint_angle(self, joint: Joint, angle: float):
        self.angles[joint.id - 1] = angle
        self._angles_synced = False

    def set_base_pose(self, vec):
        self.base_pose = np.asarray(vec, np.float64).copy()

    def set_joint_angles(self, joints: Sequence[Joint], angles):
        angles = np.asarray(angles, np.float64)
        n = len(joints)
        assert angles.size == n + (3 if self.with_base else 0)
        for j, a in zip(joints, angles[:n]):
            self.angles[j.id - 1] = a
        if self.with_base:
            self.base_pose = angles[n:n + 3].copy()
        self._angles_synced = False

    def get_joint_angles(self, joints: Sequence[Joint]) -> np.ndarray:
        out = [self.angles[j.id - 1] for j in joints]
        if self.with_base:
            out += list(self.base_pose)
        return np.array(out, np.float64)

    # -- add_new_link (src/mechanism.jl:233-267) ------------------------------
    def add_new_link(self, new_link: Link, parent: Link, pose_or_position):
        T = np.asarray(pose_or_position, np.float64)
        if T.shape == (3,):
            P = np.eye(4)
            P[:3, 3] = T
            T = P
        T16 = np.ascontiguousarray(T.T.reshape(16))
        nid = C.c_int32()
        K.check(K.lib().kin_model_add_link(self._model, parent.id, _p(T16), C.byref(nid)))
        hid = len(self.links) + 1
        assert nid.value == hid
        jid = len(self.joints) + 1
        parent.clink_ids.append(hid)
        parent.cjoint_ids.append(jid)
        jnt = Joint(new_link.name + "_joint", jid, parent.id, hid, T.copy(), "fixed", np.array([1.0, 0, 0]))
        new_link.id, new_link.pjoint_id, new_link.plink_id = hid, jid, parent.id
        new_link.cjoint_ids, new_link.clink_ids, new_link.data = [], [], {}
        self.links.append(new_link)
        self.joints.append(jnt)
        self.linkid_map[new_link.name] = hid
        self.jointid_map[jnt.name] = jid
        self.angles = np.append(self.angles, 0.0)
        self._angles_synced = False
        return new_link

    # -- batched hot path -------------------------------------------------------
    def plan(self, q_joints: Sequence[Joint], out_links: Sequence[Link] = (), jac_link: Optional[Link] = None,
             jac_joints: Optional[Sequence[Joint]] = None, with_rot: bool = True, rpy_jac: bool = False,
             zero_fill: bool = True, dtype=torch.float32, specialize=False) -> "Plan":
        """A staged evaluation program (kin_plan_create).  `specialize`: True (every kernel kind that
        applies) or a KIN_SPEC_* mask compiles it into constant-folded kernels (kin_plan_specialize)."""
        self._sync_angles()
        p = Plan(self, q_joints, out_links, jac_link, jac_joints, with_rot, rpy_jac, zero_fill, dtype)
        if specialize:
            p.specialize(0 if specialize is True else int(specialize))
        return p


class Plan:
    """A staged, device-resident evaluation program (kin_plan)."""

    def __init__(self, m: Mechanism, q_joints, out_links, jac_link, jac_joints, with_rot, rpy_jac, zero_fill,
                 dtype):
        if dtype not in _DT:
            raise TypeError("dtype must be torch.float32 or torch.float64")
        self.m, self.dtype = m, dtype
        self._q = _ids(q_joints)
        self._o = _ids(out_links)
        self._jl = 0 if jac_link is None else jac_link.id
        if jac_link is not None and jac_joints is None:
            jac_joints = q_joints
        self._j = _ids(jac_joints or [])
        flags = (K.KIN_WITH_ROT if with_rot else 0) | (K.KIN_RPY_JAC if rpy_jac else 0) | \
                (K.KIN_ZERO_FILL if zero_fill else 0)
        self.zero_fill = zero_fill
        d = K.PlanDesc(_DT[dtype], self._q.size, _p(self._q).value, self._o.size, _p(self._o).value,
                       self._jl, self._j.size, _p(self._j).value, flags)
        self._h = C.c_void_p()
        _raise_like_julia(K.lib().kin_plan_create(m._model, C.byref(d), C.byref(self._h)))
        nq, rows, cols = C.c_int32(), C.c_int32(), C.c_int32()
        K.check(K.lib().kin_plan_shape(self._h, C.byref(nq), C.byref(rows), C.byref(cols)))
        self.n_qcols, self.jac_rows, self.jac_cols = nq.value, rows.value, cols.value
        self.n_out = self._o.size
        self.device_index = _current_device_index()  # the HIP device the plan was staged on

    def __del__(self):
        if getattr(self, "_h", None) and K._lib is not None:
            K._lib.kin_plan_destroy(self._h)
            self._h = None

    def specialize(self, kernels: int = 0) -> "Plan":
        """kin_plan_specialize: compile this plan's program into constant-folded gfx950 kernels
        (hiprtc; synchronous, cached per process).  Returns self."""
        K.check(K.lib().kin_plan_specialize(self._h, int(kernels)))
        return self

    @property
    def specialized(self) -> int:
        v = C.c_uint32()
        K.check(K.lib().kin_plan_specialized(self._h, C.byref(v)))
        return v.value

    def ik_sched_stats(self) -> dict:
        """kin_plan_ik_sched_stats: counters of the two-phase IK scratch-set scheduling (tests)."""
        st = K.IkSchedStats()
        K.check(K.lib().kin_plan_ik_sched_stats(self._h, C.byref(st)))
        return {name: int(getattr(st, name)) for name, _ in K.IkSchedStats._fields_}

    def _check_q(self, Q: torch.Tensor) -> int:
        if not Q.is_cuda or Q.dtype != self.dtype or Q.dim() != 2 or Q.shape[0] != self.n_qcols:
            raise ValueError(f"Q must be a CUDA {self.dtype} tensor of shape ({self.n_qcols}, N)")
        if Q.stride(1) != 1:
            raise ValueError("Q must be configuration-contiguous (stride(1) == 1)")
        _plan_device(self, Q)
        return Q.shape[1]

    def run(self, Q: torch.Tensor, poses: Optional[torch.Tensor] = None, jac: Optional[torch.Tensor] = None,
            stream: Optional[torch.cuda.Stream] = None):
        """Evaluate N configurations; returns (poses [n_out,12,N], jac [cols,rows,N] or None). Async."""
        N = self._check_q(Q)
        dev = Q.device
        if poses is None and self.n_out:
            poses = torch.empty((self.n_out, 12, N), dtype=self.dtype, device=dev)
        if jac is None and self._jl:
            alloc = torch.zeros if not self.zero_fill else torch.empty
            jac = alloc((self.jac_cols, self.jac_rows, N), dtype=self.dtype, device=dev)
        for t, what in ((poses, "poses"), (jac, "jac")):
            if t is not None:
                _same_device(t, Q, what)
        ldp = _ld_of(poses, (self.n_out, 12, N), self.dtype) if poses is not None else N
        ldj = _ld_of(jac, (self.jac_cols, self.jac_rows, N), self.dtype) if jac is not None else N
        st = (stream or torch.cuda.current_stream(dev)).cuda_stream
        ldq = Q.stride(0) if self.n_qcols else N
        K.check(K.lib().kin_plan_run(self._h, Q.data_ptr() if self.n_qcols else None, ldq, N,
                                     poses.data_ptr() if poses is not None else None, ldp,
                                     jac.data_ptr() if jac is not None else None, ldj, st))
        return poses, jac

    def run_tiled(self, Qt: torch.Tensor, n: int, poses: Optional[torch.Tensor] = None,
                  jac: Optional[torch.Tensor] = None, stream: Optional[torch.cuda.Stream] = None):
        """kin_plan_run_tiled: the tiled-SoA layout (include/kinhip.h).  Qt is (ntiles, n_qcols, tile)
        with unit configuration stride (``tiled(Q, tile)``); outputs are (ntiles, n_out, 12, tile) and
        (ntiles, cols, rows, tile).  `n` <= ntiles * tile configurations are evaluated.  Async."""
        if not Qt.is_cuda or Qt.dtype != self.dtype or Qt.dim() != 3 or Qt.shape[1] != self.n_qcols:
            raise ValueError(f"Qt must be a CUDA {self.dtype} tensor of shape (ntiles, {self.n_qcols}, tile)")
        nt, _, tile = Qt.shape
        if Qt.stride(2) != 1 or not 0 <= n <= nt * tile:
            raise ValueError("Qt must be configuration-contiguous and hold n configurations")
        _plan_device(self, Qt)
        dev = Qt.device
        if poses is None and self.n_out:
            poses = torch.empty((nt, self.n_out, 12, tile), dtype=self.dtype, device=dev)
        if jac is None and self._jl:
            alloc = torch.zeros if not self.zero_fill else torch.empty
            jac = alloc((nt, self.jac_cols, self.jac_rows, tile), dtype=self.dtype, device=dev)

        def geom(t, shape):
            if t is None:
                return None, tile, 0
            if tuple(t.shape) != shape or t.dtype != self.dtype or not t.is_cuda or t.stride(3) != 1:
                raise ValueError(f"tiled output must be a CUDA {self.dtype} tensor of shape {shape}")
            _same_device(t, Qt, "tiled output")
            a, b = shape[1], shape[2]
            ld = t.stride(2)
            if a > 1 and t.stride(1) != b * ld:
                raise ValueError("tiled output rows must be evenly spaced")
            return t.data_ptr(), ld, t.stride(0)

        pp, ldp, tsp = geom(poses, (nt, self.n_out, 12, tile))
        jp, ldj, tsj = geom(jac, (nt, self.jac_cols, self.jac_rows, tile))
        st = (stream or torch.cuda.current_stream(dev)).cuda_stream
        K.check(K.lib().kin_plan_run_tiled(self._h, tile, Qt.data_ptr() if self.n_qcols else None, Qt.stride(1),
                                           Qt.stride(0), n, pp, ldp, tsp, jp, ldj, tsj, st))
        return poses, jac

    def ik_dls(self, targets: torch.Tensor, Q: torch.Tensor, max_iters=64, lam=1e-2, tol_pos=1e-3, tol_rot=1e-3,
               max_step=0.5, with_rot=True, restarts=0, seed=0, lanes=0, index_base=0, stream=None, Q0=None,
               damp_err=0.0):
        """Batched DLS IK in place on Q; returns (Q, iters int32 [N], err [2, N]).  `lanes`: lanes per
        target running restart attempts side by side (0 auto, which runs batches of more than one round
        of waves in two phases: attempt 0 of every target, then the other attempts of the unsolved ones;
        results identical for every value).
        `index_base`: global index of target 0 for the restart draws (a shard's offset), so a target
        set sharded over ranks solves exactly as in one process.  iters > max_iters: not converged.
        `Q0`: starting angles read from Q0 (same shape and strides as Q, not modified) and Q written
        without being read (``kin_ik_dls_batch_from``): the results of ``Q.copy_(Q0)`` + the in-place
        call, without the copy.
        `with_rot`: 0 position only, 1 (True) axis-angle residual, 2 the reference's objective
        (src/inverse_kinematics.jl:38-50: [p* - p; rpy* - rpy] with the rpy_jac Jacobian; `tol_rot`
        then bounds |d rpy| and err[1] is |d rpy|).
        `damp_err`: error-scaled damping -- each iteration solves with lam^2 + damp_err (|dp|^2 + |rot|^2)
        (Levenberg-Marquardt after Sugihara; 0: fixed lam)."""
        N = self._check_q(Q)
        if Q0 is not None:
            _same_device(Q0, Q, "Q0")
            if Q0.shape != Q.shape or Q0.stride() != Q.stride() or Q0.dtype != Q.dtype:
                raise ValueError("Q0 must have Q's shape, strides and dtype")
        if targets.shape != (12, N) or targets.dtype != self.dtype or not targets.is_contiguous():
            raise ValueError("targets must be a contiguous (12, N) tensor of the plan dtype")
        _same_device(targets, Q, "targets")
        iters = torch.empty(N, dtype=torch.int32, device=Q.device)
        err = torch.empty((2, N), dtype=self.dtype, device=Q.device)
        prm = K.IkParams(int(max_iters), float(lam), float(tol_pos), float(tol_rot), float(max_step), int(with_rot),
                         int(restarts), int(seed), int(lanes), int(index_base), float(damp_err))
        st = (stream or torch.cuda.current_stream(Q.device)).cuda_stream
        if Q0 is not None:
            K.check(K.lib().kin_ik_dls_batch_from(self._h, C.byref(prm), targets.data_ptr(), N, Q0.data_ptr(),
                                                  Q.data_ptr(), Q.stride(0), N, iters.data_ptr(), err.data_ptr(), N,
                                                  st))
        else:
            K.check(K.lib().kin_ik_dls_batch(self._h, C.byref(prm), targets.data_ptr(), N, Q.data_ptr(), Q.stride(0),
                                             N, iters.data_ptr(), err.data_ptr(), N, st))
        return Q, iters, err

    def ik_dls_trace(self, targets: torch.Tensor, Q0: torch.Tensor, max_iters=64, lam=1e-2, tol_pos=1e-3,
                     tol_rot=1e-3, max_step=0.5, with_rot=True, restarts=0, seed=0, index_base=0, stream=None,
                     damp_err=0.0):
        """``kin_ik_dls_batch_trace``: ik_dls from Q0 that also records |dp| and |rot| of every iterate ->
        (Q, iters [N], trace [max_iters + 1, 2, N]); rows of iterations a target does not reach are NaN."""
        N = self._check_q(Q0)
        if targets.shape != (12, N) or targets.dtype != self.dtype or not targets.is_contiguous():
            raise ValueError("targets must be a contiguous (12, N) tensor of the plan dtype")
        _same_device(targets, Q0, "targets")
        Q = torch.empty_like(Q0)
        iters = torch.empty(N, dtype=torch.int32, device=Q0.device)
        trace = torch.full((int(max_iters) + 1, 2, N), float("nan"), dtype=self.dtype, device=Q0.device)
        prm = K.IkParams(int(max_iters), float(lam), float(tol_pos), float(tol_rot), float(max_step), int(with_rot),
                         int(restarts), int(seed), 1, int(index_base), float(damp_err))
        st = (stream or torch.cuda.current_stream(Q0.device)).cuda_stream
        K.check(K.lib().kin_ik_dls_batch_trace(self._h, C.byref(prm), targets.data_ptr(), N, Q0.data_ptr(),
                                               Q.data_ptr(), Q.stride(0), N, iters.data_ptr(), trace.data_ptr(), N, st))
        return Q, iters, trace

    def point_ik_nakamura(self, points: torch.Tensor, Q: torch.Tensor, stream=None):
        N = self._check_q(Q)
        if points.shape != (3, N) or points.dtype != self.dtype or not points.is_contiguous():
            raise ValueError("points must be a contiguous (3, N) tensor of the plan dtype")
        _same_device(points, Q, "points")
        st = (stream or torch.cuda.current_stream(Q.device)).cuda_stream
        K.check(K.lib().kin_point_ik_nakamura_batch(self._h, points.data_ptr(), N, Q.data_ptr(), Q.stride(0), N, st))
        return Q


# ---------------------------------------------------------------------------
# URDF (src/load_urdf.jl:20-80) through the native parser
# ---------------------------------------------------------------------------
def parse_urdf(urdf_path: str, with_base: bool = False, name: Optional[str] = None) -> Mechanism:
    L = K.lib()
    u = C.c_void_p()
    K.check(L.kin_urdf_parse_file(urdf_path.encode(), C.byref(u)))
    try:
        d = K.TreeDesc()
        K.check(L.kin_urdf_tree(u, int(with_base), C.byref(d)))
        nl, nj = d.n_links, d.n_joints
        as_np = lambda ptr, n, ct: np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(n,)).copy() if n else \
            np.zeros(0)
        jt = as_np(d.joint_type, nj, C.c_int32)
        jp = as_np(d.joint_plink, nj, C.c_int32)
        jc = as_np(d.joint_clink, nj, C.c_int32)
        pose = as_np(d.joint_pose, 16 * nj, C.c_double).reshape(nj, 16)
        axis = as_np(d.joint_axis, 3 * nj, C.c_double).reshape(nj, 3)
        lo = as_np(d.joint_lower, nj, C.c_double)
        hi = as_np(d.joint_upper, nj, C.c_double)
        nm = C.c_char_p()
        links = []
        for i in range(1, nl + 1):
            K.check(L.kin_urdf_link_name(u, i, C.byref(nm)))
            has = C.c_int32()
            ext = np.zeros(3)
            org = np.zeros(16)
            K.check(L.kin_urdf_link_box(u, i, C.byref(has), _p(ext), _p(org)))
            meta = BoxMetaData(ext, org.reshape(4, 4).T.copy()) if has.value else None
            links.append(Link(nm.value.decode(), i, geometric_meta_data=meta))
        joints = []
        for j in range(nj):
            K.check(L.kin_urdf_joint_name(u, j + 1, C.byref(nm)))
            joints.append(Joint(nm.value.decode(), j + 1, int(jp[j]), int(jc[j]), pose[j].reshape(4, 4).T.copy(),
                                _JT[int(jt[j])], axis[j].copy(), float(lo[j]), float(hi[j])))
            p, c = links[jp[j] - 1], links[jc[j] - 1]
            p.cjoint_ids.append(j + 1)
            p.clink_ids.append(int(jc[j]))
            c.pjoint_id, c.plink_id = j + 1, int(jp[j])
    finally:
        L.kin_urdf_destroy(u)
    return Mechanism(links, joints, with_base=with_base, name=name or "basic")


# ---------------------------------------------------------------------------
# Julia-style free functions (src/Kinematics.jl exports)
# ---------------------------------------------------------------------------
def find_link(m: Mechanism, name):
    return m.find_link(name)


def find_joint(m: Mechanism, name):
    return m.find_joint(name)


def parent_link(m, x):
    return m.parent_link(x)


def child_link(m, joint):
    return m.child_link(joint)


def child_links(m, link):
    return m.child_links(link)


def parent_joint(m, link):
    return m.parent_joint(link)


def child_joints(m, link):
    return m.child_joints(link)


def isroot(link: Link) -> bool:
    return link.plink_id == -1


def isleaf(link: Link) -> bool:
    return len(link.clink_ids) == 0


def is_relevant(m: Mechanism, joint: Joint, link: Link) -> bool:
    return m.is_relevant(joint, link)


def set_joint_angles(m: Mechanism, joints, angles):
    m.set_joint_angles(joints, angles)


def get_joint_angles(m: Mechanism, joints):
    return m.get_joint_angles(joints)


def get_joint_angles_(m: Mechanism, joints, out: np.ndarray) -> np.ndarray:
    """``get_joint_angles!`` (src/mechanism.jl:203-221): fills `out` in place."""
    out[:] = m.get_joint_angles(joints)
    return out


def joint_angle(m: Mechanism, joint: Joint) -> float:
    """src/mechanism.jl:197."""
    return m.joint_angle(joint)


def set_joint_angle(m: Mechanism, joint: Joint, angle: float):
    """src/mechanism.jl:199-201."""
    m.set_joint_angle(joint, angle)


def add_new_link(m: Mechanism, new_link: Link, parent: Link, pose_or_position):
    return m.add_new_link(new_link, parent, pose_or_position)


def tiled(X: torch.Tensor, tile: int) -> torch.Tensor:
    """[..., N] SoA -> [ntiles, ..., tile] tiled SoA (N padded up to a whole number of tiles)."""
    n = X.shape[-1]
    nt = -(-n // tile)
    if nt * tile != n:
        X = torch.nn.functional.pad(X, (0, nt * tile - n))
    return X.reshape(*X.shape[:-1], nt, tile).movedim(-2, 0).contiguous()


def untiled(Xt: torch.Tensor, n: int) -> torch.Tensor:
    """Inverse of tiled(): [ntiles, ..., tile] -> [..., n]."""
    X = Xt.movedim(0, -2)
    return X.reshape(*X.shape[:-2], -1)[..., :n]


def _same_device(t: torch.Tensor, ref: torch.Tensor, what: str):
    """A device pointer handed to the C-ABI must live on the device of the launch (Q's): a host or
    other-GPU tensor would reach the kernel as a bad address (a GPU fault, not an error code)."""
    if not t.is_cuda or t.device != ref.device:
        raise ValueError(f"{what} must be a CUDA tensor on {ref.device} (got {t.device})")


def _current_device_index() -> int:
    try:
        return torch.cuda.current_device()
    except (RuntimeError, AssertionError):  # no HIP device: plan creation has failed before this
        return -1


def _plan_device(plan, Q: torch.Tensor):
    """A plan's program (and its specialised code) lives on the device it was staged on.  The C-ABI
    checks the *current* device; this checks the tensors too: Q on another device than the plan
    would launch the plan's module on Q's stream with pointers of another GPU (a GPU fault)."""
    if Q.device.index != plan.device_index:
        raise ValueError(f"the plan lives on cuda:{plan.device_index} but the tensors are on {Q.device}")


def _ld_of(t: torch.Tensor, shape, dtype) -> int:
    """Leading dimension of a [a][b][ld] SoA output given as a (possibly row-padded) view of shape
    `shape` = (a, b, N): configuration stride 1, rows `ld` apart (the C-ABI's ldp / ldj)."""
    if tuple(t.shape) != tuple(shape) or t.dtype != dtype or not t.is_cuda:
        raise ValueError(f"output must be a CUDA {dtype} tensor of shape {tuple(shape)}")
    a, b, n = shape
    ld = t.stride(1) if b > 1 else (t.stride(0) if a > 1 else n)
    if t.stride(2) != 1 or ld < n or (a > 1 and t.stride(0) != b * ld):
        raise ValueError("output rows must be evenly spaced with unit configuration stride")
    return ld


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("kinhip: no HIP device visible (the engine has no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


def _single_q(m: Mechanism, dev):
    q = list(m.angles) + (list(m.base_pose) if m.with_base else [])
    return torch.tensor(q, dtype=torch.float64, device=dev).reshape(-1, 1)


def get_transform(m: Mechanism, link: Link) -> np.ndarray:
    """World pose (4x4) of ``link`` at the mechanism's current angles (src/algorithm.jl:1-4)."""
    dev = _device()
    key = ("tf", link.id, len(m.joints), dev.index)
    plan = m.__dict__.setdefault("_single_plans", {}).get(key)
    if plan is None:
        plan = m.plan(m.joints, out_links=[link], dtype=torch.float64)
        m._single_plans[key] = plan
    poses, _ = plan.run(_single_q(m, dev))
    T = np.eye(4)
    T[:3, :4] = poses[0, :, 0].cpu().numpy().reshape(4, 3).T
    return T


def get_jacobian_(m: Mechanism, link: Link, joints, with_rot: bool, mat_out: np.ndarray, rpy_jac=False):
    """``get_jacobian!`` (src/algorithm.jl:83-106): writes relevant columns into mat_out."""
    dev = _device()
    key = ("jac", link.id, tuple(j.id for j in joints), bool(with_rot), bool(rpy_jac), len(m.joints), dev.index)
    plans = m.__dict__.setdefault("_single_plans", {})
    plan = plans.get(key)
    ids = list(range(1, len(m.joints) + 1))
    if plan is None:
        plan = Plan(m, ids, [], link, joints, with_rot, rpy_jac, False, torch.float64)
        plans[key] = plan
    jac = torch.as_tensor(np.ascontiguousarray(np.asarray(mat_out, np.float64).T)).to(dev).reshape(
        plan.jac_cols, plan.jac_rows, 1).contiguous()
    # the plan's Jacobian columns are `joints` (+ base); its q columns are every joint
    plan.run(_single_q(m, dev), jac=jac)
    mat_out[...] = jac[:, :, 0].cpu().numpy().T
    return mat_out


def get_jacobian(m: Mechanism, link: Link, joints, with_rot: bool, rpy_jac=False) -> np.ndarray:
    rows = 6 if with_rot else 3
    cols = len(joints) + (3 if m.with_base else 0)
    J = np.zeros((rows, cols))
    return get_jacobian_(m, link, joints, with_rot, J, rpy_jac=rpy_jac)


def get_transform_batch(m: Mechanism, links, joints, Q: torch.Tensor, poses: Optional[torch.Tensor] = None,
                        stream=None):
    """Batched get_transform: Q (len(joints)[+3], N) -> poses (len(links), 12, N).  Async.

    Runs through ``kin_get_transform_batch``: the C side keeps one plan per request in the model
    and drops them when the model changes (``set_joint_angles`` of joints outside `joints`,
    ``add_new_link``); that drop frees device memory, which synchronises the device once."""
    m._sync_angles()
    _check_q_batch(m, joints, Q)
    N = Q.shape[1]
    ids = _ids(joints)
    oids = _ids(links)
    if poses is None:
        poses = torch.empty((oids.size, 12, N), dtype=Q.dtype, device=Q.device)
    _same_device(poses, Q, "poses")
    ldp = _ld_of(poses, (oids.size, 12, N), Q.dtype)
    st = (stream or torch.cuda.current_stream(Q.device)).cuda_stream
    rc = K.lib().kin_get_transform_batch(m._model, _DT[Q.dtype], ids.size, _p(ids), Q.data_ptr(), Q.stride(0), N,
                                         oids.size, _p(oids), poses.data_ptr(), ldp, st)
    _raise_like_julia(rc)
    return poses


def get_jacobian_batch(m: Mechanism, link, joints, Q: torch.Tensor, with_rot=True, rpy_jac=False, stream=None):
    """Batched get_transform + get_jacobian (``kin_get_jacobian_batch``, cached per model like
    get_transform_batch): -> (pose (12, N), jac (cols, rows, N)), irrelevant columns zero.  Async."""
    m._sync_angles()
    _check_q_batch(m, joints, Q)
    N = Q.shape[1]
    ids = _ids(joints)
    rows = 6 if with_rot else 3
    cols = ids.size + (3 if m.with_base else 0)
    pose = torch.empty((1, 12, N), dtype=Q.dtype, device=Q.device)
    jac = torch.empty((cols, rows, N), dtype=Q.dtype, device=Q.device)
    flags = (K.KIN_WITH_ROT if with_rot else 0) | (K.KIN_RPY_JAC if rpy_jac else 0) | K.KIN_ZERO_FILL
    st = (stream or torch.cuda.current_stream(Q.device)).cuda_stream
    rc = K.lib().kin_get_jacobian_batch(m._model, _DT[Q.dtype], link.id, ids.size, _p(ids), flags, Q.data_ptr(),
                                        Q.stride(0), N, pose.data_ptr(), N, jac.data_ptr(), N, st)
    _raise_like_julia(rc)
    return pose[0], jac


def _check_q_batch(m: Mechanism, joints, Q: torch.Tensor):
    if Q.dtype not in _DT:
        raise TypeError("Q must be torch.float32 or torch.float64")
    nq = len(joints) + (3 if m.with_base else 0)
    if not Q.is_cuda or Q.dim() != 2 or Q.shape[0] != nq or Q.stride(1) != 1:
        raise ValueError(f"Q must be a configuration-contiguous CUDA tensor of shape ({nq}, N)")


def _raise_like_julia(rc):
    if rc != K.KIN_OK:
        msg = K.lib().kin_last_error().decode()
        raise K.error_class(rc)(msg) if rc in (K.KIN_E_KEY, K.KIN_E_METHOD) else K.KinError(rc, msg)


_SINGLE_PLAN_CAP = 16


def _cached_plan(m: Mechanism, key, make, joints=()):
    """Per-mechanism cache of the single-configuration convenience plans, keyed by the request, the
    mechanism state they bake in -- the angles of the joints the plan does NOT take as batch columns
    (the batched ones come in through Q) and the tree size -- and the device.  Least recently used
    plans beyond _SINGLE_PLAN_CAP are dropped, so a loop of IK calls that moves the batched joints
    reuses one plan and a loop that moves other joints does not grow device memory without bound."""
    batched = np.zeros(len(m.angles), bool)
    batched[[j.id - 1 for j in joints]] = True
    key = key + (np.where(batched, 0.0, m.angles).tobytes(), len(m.joints), torch.cuda.current_device())
    plans = m.__dict__.setdefault("_single_plans", {})
    p = plans.pop(key, None)
    if p is None:
        p = make()
    plans[key] = p  # most recently used last
    while len(plans) > _SINGLE_PLAN_CAP:
        plans.pop(next(iter(plans)))
    return p


def translation(T) -> np.ndarray:
    """src/transform.jl:42: the translation of a 4x4 transform."""
    return np.asarray(T, np.float64)[:3, 3].copy()


def rotation(T) -> np.ndarray:
    """src/transform.jl:43: the 3x3 rotation of a 4x4 transform."""
    return np.asarray(T, np.float64)[:3, :3].copy()


def Transform(rot=None, trans=None) -> np.ndarray:
    """src/transform.jl:16-31: a 4x4 homogeneous transform from a 3x3 rotation and/or a translation
    (identity parts where omitted; ``zero(Transform)`` is the identity, :50-52)."""
    T = np.eye(4)
    if rot is not None:
        T[:3, :3] = np.asarray(rot, np.float64)
    if trans is not None:
        T[:3, 3] = np.asarray(trans, np.float64)
    return T


def rpy(T) -> np.ndarray:
    """RotZYX angles [roll, pitch, yaw] of a 4x4 (src/transform.jl:45-48)."""
    R = np.asarray(T)[:3, :3]
    t1 = math.atan2(R[1, 0], R[0, 0])
    c1, s1 = math.cos(t1), math.sin(t1)
    t2 = math.atan2(-R[2, 0], R[1, 0] * s1 + R[0, 0] * c1)
    t3 = math.atan2(R[0, 2] * s1 - R[1, 2] * c1, R[1, 1] * c1 - R[0, 1] * s1)
    return np.array([t3, t2, t1])


def point_inverse_kinematics_nakamura(m: Mechanism, link: Link, joints, point_desired) -> np.ndarray:
    """src/algorithm.jl:116-131 on the GPU (batch of one); returns the angles."""
    dev = _device()
    m._sync_angles()
    plan = _cached_plan(m, ("nakamura", link.id, tuple(j.id for j in joints)),
                        lambda: m.plan(joints, jac_link=link, jac_joints=joints, with_rot=False, dtype=torch.float64),
                        joints)
    Q = torch.tensor([m.angles[j.id - 1] for j in joints], dtype=torch.float64, device=dev).reshape(-1, 1)
    pts = torch.tensor(np.asarray(point_desired, np.float64), device=dev).reshape(3, 1).contiguous()
    plan.point_ik_nakamura(pts, Q)
    return Q[:, 0].cpu().numpy()


def inverse_kinematics_(m: Mechanism, link: Link, joints, target_pose, sscc=None, sdf=None, use_bistage=True,
                        ftol=1e-5, with_rot=True, max_iters=200, lam=1e-2, max_step=0.5, solver="DLS"):
    """``inverse_kinematics!`` (src/inverse_kinematics.jl:1-30) -> (q, status); sets the mechanism's angles.

    Without ``sscc`` / ``sdf`` (src/inverse_kinematics.jl:23-30): the DLS kernel on the reference's
    objective (f_objective: |[p* - p; rpy* - rpy]|^2, kin_ik_params.with_rot = 2), stopped by the
    reference's ``ftol_abs`` rule (NLopt stops when one step changes the objective by less than
    ftol), checked after every step on the objective of every iterate (kin_ik_dls_batch_trace: one
    launch of max_iters steps), the stopping iterate k then one launch of k steps from the starting
    angles.  Status ``:FTOL_REACHED`` when that rule
    stopped it, ``:MAXEVAL_REACHED`` after ``max_iters`` steps.

    With ``sscc`` and ``sdf`` (src/inverse_kinematics.jl:1-21): the collision-aware form.  Stage 1
    (``use_bistage``) is the collision-free solve above; stage 2 solves the reference's objective
    subject to the sphere distances of ``IneqConst(sscc, joints, sdf, 1, 0.02)`` and the joint limits:
    by default on the GPU (``solver="DLS"``: the batched kin_ik_coll_batch kernel on a batch of one,
    ``kinhip.CollisionIKPlan`` for many targets), or with SciPy's SLSQP on the host (``solver="SLSQP"``;
    the reference uses NLopt's LD_SLSQP) over GPU evaluations.  See ``planning.collision_aware_ik``.
    """
    if (sscc is None) != (sdf is None):
        raise TypeError("inverse_kinematics_: pass both sscc and sdf (collision-aware form) or neither")
    if sscc is not None:
        from .planning import collision_aware_ik
        return collision_aware_ik(m, link, joints, target_pose, sscc, sdf, use_bistage=use_bistage, ftol=ftol,
                                  with_rot=with_rot, max_iters=max_iters, lam=lam, max_step=max_step, solver=solver)
    return _dls_ik_ftol(m, link, joints, target_pose, ftol, with_rot, max_iters, lam, max_step)


def _dls_ik_ftol(m: Mechanism, link: Link, joints, target_pose, ftol, with_rot, max_iters, lam, max_step):
    dev = _device()
    m._sync_angles()
    plan = _cached_plan(m, ("ik", link.id, tuple(j.id for j in joints)),
                        lambda: m.plan(joints, out_links=[link], jac_link=link, jac_joints=joints, with_rot=True,
                                       dtype=torch.float64), joints)
    Q0 = torch.tensor(m.get_joint_angles(joints), dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    T = np.asarray(target_pose, np.float64)
    tgt = torch.tensor(T[:3, :4].T.reshape(12), device=dev).reshape(12, 1).contiguous()
    # the reference's objective (with_rot = 2: |[p* - p; rpy* - rpy]|^2, src/inverse_kinematics.jl:38-50)
    kw = dict(lam=lam, tol_pos=0.0, tol_rot=0.0, max_step=max_step, with_rot=2 if with_rot else 0)

    # every iterate's objective from one launch of max_iters steps (kin_ik_dls_batch_trace), then the
    # stopping iterate k from a launch of k steps: O(max_iters) steps (the active set the
    # solver carries between steps lives inside the kernel, so an iterate is a launch from Q0)
    M = int(max_iters)
    _, _, tr = plan.ik_dls_trace(tgt, Q0, max_iters=M, **kw)
    tr = tr[:, :, 0].double().cpu().numpy()
    f = tr[:, 0] ** 2 + tr[:, 1] ** 2  # f_objective |[p* - p; rpy* - rpy]|^2 of iterates 0 .. M
    status, k = ":MAXEVAL_REACHED", M
    for kk in range(1, M + 1):
        if abs(f[kk - 1] - f[kk]) < ftol:
            status, k = ":FTOL_REACHED", kk
            break
    Q = torch.empty_like(Q0)
    plan.ik_dls(tgt, Q, max_iters=k, Q0=Q0, **kw)
    q = Q[:, 0].cpu().numpy()
    m.set_joint_angles(joints, q)
    return q, status
