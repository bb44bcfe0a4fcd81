"""Swept-sphere collision against box SDFs (src/sdf.jl, src/collision.jl) on the GPU.

Mirrors the reference names: ``BoxSDF(pose, width)``, ``UnionSDF(sdfs)`` /
``UnionSDF(mechanism)`` (one box per link with box collision geometry,
src/sdf.jl:82-97), ``SweptSphereCollisionChecker(mech)``,
``compute_coll_dists`` / ``compute_coll_dists_and_grads`` (single
configuration) and the batched ``CollisionPlan``.  Spheres are links added
with ``add_new_link`` exactly as ``add_coll_links`` does
(src/collision.jl:39-49); the sphere geometry itself comes from the caller
(``add_coll_sphere``): the reference derives it from mesh files with
skrobot + trimesh, which are not available here.
"""
from __future__ import annotations

import ctypes as C
import itertools
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib as K
from .mechanism import (Link, Mechanism, Plan, _current_device_index, _device, _i32, _ld_of, _p, _plan_device,
                        _same_device, get_transform)

_DT = {torch.float32: K.KIN_F32, torch.float64: K.KIN_F64}
_uid = itertools.count()


class BoxSDF:
    """src/sdf.jl:48-74: a box of full widths `width` at world pose `pose` (4x4)."""

    def __init__(self, pose, width):
        self.pose = np.asarray(pose, np.float64).reshape(4, 4)
        self.width = np.asarray(width, np.float64).reshape(3)

    def __call__(self, p):  # host convenience (the GPU path is kin_coll_batch)
        R, t = self.pose[:3, :3], self.pose[:3, 3]
        q = np.abs(R.T @ (np.asarray(p, np.float64) - t)) - 0.5 * self.width
        return float(np.linalg.norm(np.maximum(q, 0.0)) + min(q.max(), 0.0))


class UnionSDF:
    """src/sdf.jl:76-119: min over boxes.  ``UnionSDF(mech)`` uses the mechanism's current angles."""

    def __init__(self, sdfs_or_mech):
        if isinstance(sdfs_or_mech, Mechanism):
            m = sdfs_or_mech
            boxes = []
            for l in m.links:
                meta = l.geometric_meta_data
                if meta is not None and hasattr(meta, "extents"):
                    boxes.append(BoxSDF(get_transform(m, l) @ meta.origin, meta.extents))
            sdfs = boxes
        else:
            sdfs = list(sdfs_or_mech)
        if not sdfs:
            raise ValueError("UnionSDF needs at least one box")
        self.sdfs = sdfs
        P = np.ascontiguousarray(np.array([b.pose.T.reshape(16) for b in sdfs], np.float64).reshape(-1))
        W = np.ascontiguousarray(np.array([b.width for b in sdfs], np.float64).reshape(-1))
        self._h = C.c_void_p()
        K.check(K.lib().kin_sdf_create_boxes(len(sdfs), _p(P), _p(W), C.byref(self._h)))
        self.device_index = _current_device_index()

    def __del__(self):
        if getattr(self, "_h", None) and K._lib is not None:
            K._lib.kin_sdf_destroy(self._h)
            self._h = None

    def __call__(self, p):
        return min(b(p) for b in self.sdfs)


class AttachedUnionSDF:
    """``UnionSDF(mech)`` (src/sdf.jl:82-97) that keeps following the scene mechanism: one BoxSDF per link
    with box collision geometry, attached to that link (attach_to_link, :43-46), its world pose
    get_transform(scene, link) * origin (:14-32) evaluated on the device for every sample
    (kin_sdf_create_attached).  `joints` (+ the scene's planar base when it has with_base) are the scene
    columns of ``CollisionPlan.run(..., scene_q=...)``: one column vector for the whole batch, or one per
    sample (e.g. a door-angle sweep in one launch).  Other scene joints stay at the scene's current angles."""

    def __init__(self, scene: Mechanism, joints=()):
        scene._sync_angles()
        links = [l for l in scene.links if l.geometric_meta_data is not None and hasattr(l.geometric_meta_data, "extents")]
        if not links:
            raise ValueError("AttachedUnionSDF: the scene has no box collision geometry")
        self.scene, self.joints = scene, list(joints)
        self.links = links
        jids = _i32([j.id for j in self.joints])
        lids = _i32([l.id for l in links])
        org = np.ascontiguousarray(np.array([np.asarray(l.geometric_meta_data.origin, np.float64).T.reshape(16)
                                             for l in links]).reshape(-1))
        wid = np.ascontiguousarray(np.array([l.geometric_meta_data.extents for l in links], np.float64).reshape(-1))
        self.n_scene_cols = len(self.joints) + (3 if scene.with_base else 0)
        self._h = C.c_void_p()
        K.check(K.lib().kin_sdf_create_attached(scene._model, jids.size, _p(jids) if jids.size else None, lids.size,
                                                _p(lids), _p(org), _p(wid), C.byref(self._h)))
        self.device_index = _current_device_index()

    def __del__(self):
        if getattr(self, "_h", None) and K._lib is not None:
            K._lib.kin_sdf_destroy(self._h)
            self._h = None


class SweptSphereCollisionChecker:
    """src/collision.jl:32-49: spheres are fixed child links of the mechanism's links."""

    def __init__(self, mech: Mechanism):
        self.mech = mech
        self.sphere_links: list = []
        self.sphere_radii: list = []

    def add_coll_sphere(self, link: Link, center, radius: float) -> Link:
        sl = Link(f"sphere_{next(_uid)}", link_type="CollSphere")
        self.mech.add_new_link(sl, link, np.asarray(center, np.float64))
        self.sphere_links.append(sl)
        self.sphere_radii.append(float(radius))
        return sl

    def plan(self, joints, dtype=torch.float32, specialize=False) -> "CollisionPlan":
        """kin_coll_plan_create; `specialize=True` also compiles it (kin_plan_specialize)."""
        p = CollisionPlan(self, joints, dtype)
        return p.specialize() if specialize else p


class CollisionPlan:
    def __init__(self, sscc: SweptSphereCollisionChecker, joints, dtype):
        m = sscc.mech
        m._sync_angles()
        self.dtype = dtype
        self.n_sph = len(sscc.sphere_links)
        self.n_dof = len(joints) + (3 if m.with_base else 0)
        self._q = _i32([j.id for j in joints])
        self._s = _i32([l.id for l in sscc.sphere_links])
        self._r = np.ascontiguousarray(np.asarray(sscc.sphere_radii, np.float64))
        d = K.CollDesc(_DT[dtype], self._q.size, _p(self._q).value, self._s.size, _p(self._s).value, None,
                       _p(self._r).value)
        self._h = C.c_void_p()
        K.check(K.lib().kin_coll_plan_create(m._model, C.byref(d), C.byref(self._h)))
        self.device_index = _current_device_index()

    def __del__(self):
        if getattr(self, "_h", None) and K._lib is not None:
            K._lib.kin_plan_destroy(self._h)
            self._h = None

    def specialize(self) -> "CollisionPlan":
        """kin_plan_specialize(KIN_SPEC_COLL): chain + spheres compiled as constants (boxes stay data)."""
        K.check(K.lib().kin_plan_specialize(self._h, K.KIN_SPEC_COLL))
        return self

    def specialize_scene(self, sdf: "AttachedUnionSDF") -> "CollisionPlan":
        """kin_plan_specialize_scene: also compile this plan's scene kernels with `sdf`'s tables (groups,
        scene steps, boxes) as constants; later ``run(sdf, ..., scene_q=...)`` calls use them.  Returns self."""
        if not isinstance(sdf, AttachedUnionSDF):
            raise TypeError("specialize_scene needs an AttachedUnionSDF")
        K.check(K.lib().kin_plan_specialize_scene(self._h, sdf._h))
        return self

    @property
    def specialized(self) -> int:
        v = C.c_uint32()
        K.check(K.lib().kin_plan_specialized(self._h, C.byref(v)))
        return v.value

    def run(self, sdf: UnionSDF, Q: torch.Tensor, dists=True, grads=False, min_dist=False,
            truncation=float("inf"), stream=None, scene_q: Optional[torch.Tensor] = None):
        """-> (dists [n_sph, N] | None, grads [n_sph, n_dof, N] | None, min_dist [N] | None). Async.
        `dists` / `grads` may also be preallocated (row-padded) output views of those shapes.
        With an ``AttachedUnionSDF``: `scene_q` = its scene columns, (n_scene_cols, N) per sample or
        (n_scene_cols,) for the whole batch (kin_coll_batch_scene)."""
        if isinstance(sdf, AttachedUnionSDF):
            return self._run_scene(sdf, Q, dists, grads, min_dist, truncation, stream, scene_q)
        if Q.dtype != self.dtype or not Q.is_cuda or Q.dim() != 2 or Q.shape[0] != self.n_dof or Q.stride(1) != 1:
            raise ValueError(f"Q must be a CUDA {self.dtype} tensor of shape ({self.n_dof}, N)")
        N = Q.shape[1]
        _plan_device(self, Q)
        _plan_device(sdf, Q)
        dev = Q.device
        D = dists if isinstance(dists, torch.Tensor) else (
            torch.empty((self.n_sph, N), dtype=self.dtype, device=dev) if dists else None)
        G = grads if isinstance(grads, torch.Tensor) else (
            torch.empty((self.n_sph, self.n_dof, N), dtype=self.dtype, device=dev) if grads else None)
        Mn = torch.empty(N, dtype=self.dtype, device=dev) if min_dist else None
        for t, what in ((D, "dists"), (G, "grads")):
            if t is not None:
                _same_device(t, Q, what)
        ldd = _ld_of(D.unsqueeze(0), (1, self.n_sph, N), self.dtype) if D is not None else N
        ldg = _ld_of(G, (self.n_sph, self.n_dof, N), self.dtype) if G is not None else N
        st = (stream or torch.cuda.current_stream(dev)).cuda_stream
        ptr = lambda t: t.data_ptr() if t is not None else None
        K.check(K.lib().kin_coll_batch(self._h, sdf._h, float(truncation), Q.data_ptr(), Q.stride(0), N, ptr(D), ldd,
                                       ptr(G), ldg, ptr(Mn), st))
        return D, G, Mn


def _run_scene(self, sdf, Q, dists, grads, min_dist, truncation, stream, scene_q):
    if Q.dtype != self.dtype or not Q.is_cuda or Q.dim() != 2 or Q.shape[0] != self.n_dof or Q.stride(1) != 1:
        raise ValueError(f"Q must be a CUDA {self.dtype} tensor of shape ({self.n_dof}, N)")
    N = Q.shape[1]
    _plan_device(self, Q)
    _plan_device(sdf, Q)
    if scene_q is None:
        raise ValueError("an AttachedUnionSDF needs scene_q (its scene joint values)")
    if scene_q.dtype != self.dtype:
        raise ValueError("scene_q must have the plan dtype")
    _same_device(scene_q, Q, "scene_q")
    if scene_q.dim() == 1:
        if scene_q.shape[0] != sdf.n_scene_cols or not scene_q.is_contiguous():
            raise ValueError(f"scene_q must hold {sdf.n_scene_cols} values")
        lds = 0
    else:
        if scene_q.shape != (sdf.n_scene_cols, N) or scene_q.stride(1) != 1:
            raise ValueError(f"scene_q must be ({sdf.n_scene_cols}, N) with unit sample stride")
        lds = scene_q.stride(0)
    dev = Q.device
    # (preallocated, row-padded output views as in run)
    D = dists if isinstance(dists, torch.Tensor) else (
        torch.empty((self.n_sph, N), dtype=self.dtype, device=dev) if dists else None)
    G = grads if isinstance(grads, torch.Tensor) else (
        torch.empty((self.n_sph, self.n_dof, N), dtype=self.dtype, device=dev) if grads else None)
    Mn = torch.empty(N, dtype=self.dtype, device=dev) if min_dist else None
    for t, what in ((D, "dists"), (G, "grads")):
        if t is not None:
            _same_device(t, Q, what)
    ldd = _ld_of(D.unsqueeze(0), (1, self.n_sph, N), self.dtype) if D is not None else N
    ldg = _ld_of(G, (self.n_sph, self.n_dof, N), self.dtype) if G is not None else N
    st = (stream or torch.cuda.current_stream(dev)).cuda_stream
    ptr = lambda t: t.data_ptr() if t is not None else None
    K.check(K.lib().kin_coll_batch_scene(self._h, sdf._h, float(truncation), Q.data_ptr(), Q.stride(0),
                                         scene_q.data_ptr() if scene_q.numel() else None, lds, N, ptr(D), ldd, ptr(G),
                                         ldg, ptr(Mn), st))
    return D, G, Mn


CollisionPlan._run_scene = _run_scene


class CollisionIKPlan(Plan):
    """kin_coll_ik_plan_create: the IK plan of `link` over `joints` with the tree of the target link and the
    checker's spheres (on any chain: both arms, torso, head) -- both stages of inverse_kinematics!(m, link,
    joints, target, sscc, sdf; use_bistage) (src/inverse_kinematics.jl:1-21) for many targets per launch
    (``solve``).  It is also an ordinary IK plan (``ik_dls``)."""

    def __init__(self, sscc: SweptSphereCollisionChecker, link: Link, joints, dtype=torch.float32):
        m = sscc.mech
        m._sync_angles()
        if dtype not in _DT:
            raise TypeError("dtype must be torch.float32 or torch.float64")
        self.m, self.dtype, self.sscc, self.link = m, dtype, sscc, link
        self._q = _i32([j.id for j in joints])
        self._o = _i32([link.id])
        self._jl = link.id
        self._j = self._q
        self.zero_fill = True
        self._s = _i32([l.id for l in sscc.sphere_links])
        self._r = np.ascontiguousarray(np.asarray(sscc.sphere_radii, np.float64))
        d = K.CollDesc(_DT[dtype], self._q.size, _p(self._q).value, self._s.size,
                       _p(self._s).value if self._s.size else None, None, _p(self._r).value if self._s.size else None)
        self._h = C.c_void_p()
        K.check(K.lib().kin_coll_ik_plan_create(m._model, C.byref(d), link.id, C.byref(self._h)))
        nq, rows, cols = C.c_int32(), C.c_int32(), C.c_int32()
        K.check(K.lib().kin_plan_shape(self._h, C.byref(nq), C.byref(rows), C.byref(cols)))
        self.n_qcols, self.jac_rows, self.jac_cols = nq.value, rows.value, cols.value
        self.n_out = 1
        self.n_sph = self._s.size
        self.device_index = _current_device_index()

    def specialize(self, kernels: int = 0) -> "CollisionIKPlan":
        """kin_plan_specialize (default: both stages' kernels over static and attached unions,
        KIN_SPEC_IK | KIN_SPEC_IK_COLL | KIN_SPEC_IK_COLL_SCENE)."""
        K.check(K.lib().kin_plan_specialize(
            self._h, int(kernels) or (K.KIN_SPEC_IK | K.KIN_SPEC_IK_COLL | K.KIN_SPEC_IK_COLL_SCENE)))
        return self

    def ik_coll(self, sdf, targets: torch.Tensor, Q: torch.Tensor, Q0: Optional[torch.Tensor] = None,
                margin=0.02, band=0.0, weight=1.0, feas=1e-6, max_iters=64, lam=1e-2, tol_pos=1e-3, tol_rot=1e-3,
                max_step=0.5, with_rot=2, restarts=0, seed=0, lanes=0, index_base=0, stream=None,
                scene_q: Optional[torch.Tensor] = None, Q_alt: Optional[torch.Tensor] = None):
        """Stage 2 alone (kin_ik_coll_batch): from Q0 (or Q in place) -> (Q, iters [N], err [3, N]:
        |dp|, |rot|, min sphere distance).  iters > max_iters: not converged (Q, err: the attempt with the
        best end state).  `lanes`: 0 = auto (restart attempts side by side and spheres shared out over lanes
        for small batches), 1 = attempts in sequence on one lane; the results do not depend on it.
        With an ``AttachedUnionSDF`` (kin_ik_coll_batch_scene): `scene_q` = its scene columns per target
        (n_scene_cols, N) or one vector (n_scene_cols,) for the batch.  `Q_alt` (Q's shape and strides;
        kin_ik_coll_batch_alt): the restart origin -- attempt 1 starts its joints from it instead of a draw,
        and every restart its base."""
        N = self._check_q(Q)
        _plan_device(sdf, Q)
        for name, X in (("Q0", Q0), ("Q_alt", Q_alt)):
            if X is not None:
                _same_device(X, Q, name)
                if X.shape != Q.shape or X.stride() != Q.stride() or X.dtype != Q.dtype:
                    raise ValueError(f"{name} must have Q's shape, strides and dtype")
        if targets.shape != (12, N) or targets.dtype != self.dtype or not targets.is_contiguous():
            raise ValueError("targets must be a contiguous (12, N) tensor of the plan dtype")
        _same_device(targets, Q, "targets")
        iters = torch.empty(N, dtype=torch.int32, device=Q.device)
        err = torch.empty((3, N), dtype=self.dtype, device=Q.device)
        prm = K.IkParams(int(max_iters), float(lam), float(tol_pos), float(tol_rot), float(max_step), int(with_rot),
                         int(restarts), int(seed), int(lanes), int(index_base))
        cp = K.IkCollParams(float(margin), float(band), float(weight), float(feas))
        st = (stream or torch.cuda.current_stream(Q.device)).cuda_stream
        q0p = (Q0 if Q0 is not None else Q).data_ptr()
        scene_p, lds = None, 0
        if isinstance(sdf, AttachedUnionSDF):
            if scene_q is None:
                raise ValueError("an AttachedUnionSDF needs scene_q (its scene joint values)")
            if scene_q.dtype != self.dtype:
                raise ValueError("scene_q must have the plan dtype")
            _same_device(scene_q, Q, "scene_q")
            if scene_q.dim() == 1:
                if scene_q.shape[0] != sdf.n_scene_cols or not scene_q.is_contiguous():
                    raise ValueError(f"scene_q must hold {sdf.n_scene_cols} values")
                lds = 0
            else:
                if scene_q.shape != (sdf.n_scene_cols, N) or scene_q.stride(1) != 1:
                    raise ValueError(f"scene_q must be ({sdf.n_scene_cols}, N) with unit target stride")
                lds = scene_q.stride(0)
            scene_p = scene_q.data_ptr() if scene_q.numel() else None
        elif scene_q is not None:
            raise ValueError("scene_q is only for an AttachedUnionSDF")
        if Q_alt is not None:
            K.check(K.lib().kin_ik_coll_batch_alt(self._h, sdf._h, C.byref(prm), C.byref(cp), targets.data_ptr(), N,
                                                  scene_p, lds, q0p, Q_alt.data_ptr(), Q.data_ptr(), Q.stride(0), N,
                                                  iters.data_ptr(), err.data_ptr(), N, st))
        elif isinstance(sdf, AttachedUnionSDF):
            K.check(K.lib().kin_ik_coll_batch_scene(self._h, sdf._h, C.byref(prm), C.byref(cp), targets.data_ptr(), N,
                                                    scene_p, lds, q0p, Q.data_ptr(), Q.stride(0), N, iters.data_ptr(),
                                                    err.data_ptr(), N, st))
        else:
            K.check(K.lib().kin_ik_coll_batch(self._h, sdf._h, C.byref(prm), C.byref(cp), targets.data_ptr(), N, q0p,
                                              Q.data_ptr(), Q.stride(0), N, iters.data_ptr(), err.data_ptr(), N, st))
        return Q, iters, err

    def solve(self, sdf, targets: torch.Tensor, Q0: torch.Tensor, use_bistage=True, margin=0.02,
              with_rot=2, max_iters=64, restarts=3, seed=0, index_base=0, stream=None, alt_start=True, **kw):
        """Both stages on the device, no host round trip: stage 1 (use_bistage) = the collision-free
        DLS (kin_ik_dls_batch_from, the seeds read from Q0), stage 2 = kin_ik_coll_batch from its
        result (src/inverse_kinematics.jl:1-21).  -> (Q, iters, err [3, N]) of stage 2.
        alt_start (with use_bistage and restarts >= 1): stage 2's restarts start from Q0, the pose stage 1
        started from (kin_ik_coll_batch_alt: attempt 1 at Q0, later attempts drawn joints on Q0's base),
        instead of from stage 1's answer, whose base stage 1 has moved."""
        Q = torch.empty_like(Q0)
        ik_kw = {k: v for k, v in kw.items() if k in ("lam", "tol_pos", "tol_rot", "max_step")}
        if use_bistage:
            self.ik_dls(targets, Q, Q0=Q0, max_iters=max_iters, restarts=restarts, seed=seed, with_rot=with_rot,
                        index_base=index_base, stream=stream, **ik_kw)
            return self.ik_coll(sdf, targets, Q, margin=margin, with_rot=with_rot, max_iters=max_iters,
                                restarts=restarts, seed=seed, index_base=index_base, stream=stream,
                                Q_alt=Q0 if alt_start else None, **kw)
        return self.ik_coll(sdf, targets, Q, Q0=Q0, margin=margin, with_rot=with_rot, max_iters=max_iters,
                            restarts=restarts, seed=seed, index_base=index_base, stream=stream, **kw)


def compute_coll_dists_(sscc: SweptSphereCollisionChecker, joints, sdf: UnionSDF, out_vals: np.ndarray):
    """``compute_coll_dists!`` (src/collision.jl:51-58): fills out_vals in place."""
    out_vals[:] = compute_coll_dists(sscc, joints, sdf)
    return out_vals


def compute_coll_dists_and_grads_(sscc: SweptSphereCollisionChecker, joints, sdf: UnionSDF, out_vals: np.ndarray,
                                  out_grads: np.ndarray, truncation_dist=float("inf")):
    """``compute_coll_dists_and_grads!`` (src/collision.jl:67-94): out_vals [n_sph], out_grads [n_dof, n_sph]."""
    v, g = compute_coll_dists_and_grads(sscc, joints, sdf, truncation_dist=truncation_dist)
    out_vals[:] = v
    out_grads[:, :] = g
    return out_vals, out_grads


def compute_swept_sphere(link: Link):
    """src/collision.jl:16-30 -> (centers [(x, y, z)], radii).  The reference fits spheres to the
    link's collision mesh with skrobot + trimesh (offline-unavailable); this returns the
    build-defined table entry (FETCH_LINK_SPHERES), or no spheres for a link it does not cover."""
    entries = FETCH_LINK_SPHERES.get(link.name, [])
    return [np.asarray(c, np.float64) for c, _ in entries], [float(r) for _, r in entries]


def compute_coll_dists(sscc: SweptSphereCollisionChecker, joints, sdf: UnionSDF) -> np.ndarray:
    """src/collision.jl:60-65 at the mechanism's current angles (GPU, batch of one)."""
    d, _ = compute_coll_dists_and_grads(sscc, joints, sdf, with_grad=False)
    return d


def compute_coll_dists_and_grads(sscc: SweptSphereCollisionChecker, joints, sdf: UnionSDF,
                                 truncation_dist=float("inf"), with_grad=True):
    """src/collision.jl:96-103: (vals [n_sph], grads [n_dof, n_sph])."""
    m = sscc.mech
    if not sscc.sphere_links:  # (the reference's own PR2 test builds a checker without spheres)
        n_dof = len(joints) + (3 if m.with_base else 0)
        return np.zeros(0), (np.zeros((n_dof, 0)) if with_grad else None)
    dev = _device()
    plan = CollisionPlan(sscc, joints, torch.float64)
    Q = torch.tensor(m.get_joint_angles(joints), dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    D, G, _ = plan.run(sdf, Q, dists=True, grads=with_grad, truncation=truncation_dist)
    vals = D[:, 0].cpu().numpy()
    return vals, (G[:, :, 0].cpu().numpy().T if with_grad else None)


# Build-defined sphere approximation of the Fetch arm (the reference computes
# spheres from collision meshes with skrobot/trimesh: unavailable offline).
# (link, centre in the link frame, radius); the arm links extend along +x.
FETCH_ARM_SPHERES = [
    ("shoulder_pan_link", (0.06, 0.0, 0.06), 0.08),
    ("shoulder_lift_link", (0.05, 0.0, 0.0), 0.07),
    ("shoulder_lift_link", (0.15, 0.0, 0.0), 0.07),
    ("upperarm_roll_link", (0.05, 0.0, 0.0), 0.065),
    ("upperarm_roll_link", (0.12, 0.0, 0.0), 0.065),
    ("elbow_flex_link", (0.05, 0.0, 0.0), 0.06),
    ("elbow_flex_link", (0.13, 0.0, 0.0), 0.06),
    ("forearm_roll_link", (0.05, 0.0, 0.0), 0.055),
    ("forearm_roll_link", (0.12, 0.0, 0.0), 0.055),
    ("wrist_flex_link", (0.05, 0.0, 0.0), 0.05),
    ("wrist_flex_link", (0.10, 0.0, 0.0), 0.05),
    ("wrist_roll_link", (0.06, 0.0, 0.0), 0.05),
    ("gripper_link", (-0.05, 0.0, 0.0), 0.05),
    ("gripper_link", (0.0, 0.0, 0.0), 0.045),
]


# The same for the PR2 arms of tests/golden/pr2_two_arms.urdf: the links of rarm_collision_links /
# larm_collision_links (src/models.jl:39-57), upper arm and forearm along +x, palm and fingers.
PR2_ARM_SPHERES = [
    (side + name, c, r) for side in ("r_", "l_") for name, c, r in (
        ("upper_arm_link", (0.1, 0.0, 0.0), 0.1), ("upper_arm_link", (0.26, 0.0, 0.0), 0.085),
        ("forearm_link", (0.1, 0.0, 0.0), 0.07), ("forearm_link", (0.22, 0.0, 0.0), 0.06),
        ("gripper_palm_link", (0.06, 0.0, 0.0), 0.055),
        ("gripper_r_finger_link", (0.04, 0.0, 0.0), 0.025), ("gripper_l_finger_link", (0.04, 0.0, 0.0), 0.025))
]
PR2_RARM_JOINTS = ["r_shoulder_pan_joint", "r_shoulder_lift_joint", "r_upper_arm_roll_joint", "r_elbow_flex_joint",
                   "r_forearm_roll_joint", "r_wrist_flex_joint", "r_wrist_roll_joint"]  # src/models.jl:13-24
PR2_LARM_JOINTS = [n.replace("r_", "l_", 1) for n in PR2_RARM_JOINTS]                  # src/models.jl:26-37
# reset_manip_pose (src/models.jl:59-70): rarm, larm (degrees), torso
PR2_MANIP_POSE = ([-75., 50., -110., -110., 20., -10., -10.], [75., 50., 110., -110., -20., -10., -10.], 0.3)


# per-link table used by add_coll_links (the arm spheres above plus the torso column)
FETCH_LINK_SPHERES: dict = {}
for _name, _c, _r in FETCH_ARM_SPHERES + [("torso_lift_link", (-0.08, 0.0, z), 0.16) for z in (0.15, 0.35, 0.55)]:
    FETCH_LINK_SPHERES.setdefault(_name, []).append((_c, _r))


def add_coll_links(sscc: SweptSphereCollisionChecker, coll_link: Link, spheres=None):
    """src/collision.jl:39-49: attach the swept spheres of `coll_link` as CollSphere links.
    The reference computes them from the link's collision mesh (skrobot + trimesh, offline-
    unavailable); here they come from `spheres` [(centre, radius), ...] or the build-defined
    FETCH_LINK_SPHERES table (KeyError for a link it does not cover)."""
    for c, r in (spheres if spheres is not None else FETCH_LINK_SPHERES[coll_link.name]):
        sscc.add_coll_sphere(coll_link, c, r)
    return sscc


def add_fetch_arm_spheres(sscc: SweptSphereCollisionChecker):
    for name, c, r in FETCH_ARM_SPHERES:
        sscc.add_coll_sphere(sscc.mech.find_link(name), c, r)
    return sscc


def fridge_sdf(fridge: Mechanism, door_angle=2.0, base=(1.2, 0.0, 0.0)) -> UnionSDF:
    """The fridge scene of test/test_inverse_kinematics.jl:52-70 (door at 2.0 rad, base (1.2, 0, 0))."""
    door = fridge.find_joint("door_joint")
    fridge.set_joint_angles([door], [door_angle, *base])
    return UnionSDF(fridge)
