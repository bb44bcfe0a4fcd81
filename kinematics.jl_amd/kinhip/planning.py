"""Trajectory-optimisation constraints over waypoints (src/planning.jl) on the GPU.

SURVEY.md 8f row f3.  The constraint evaluations -- the serial inner loop of
``plan_trajectory`` in the reference (one ``set_joint_angles`` +
``compute_coll_dists_and_grads`` per waypoint, src/planning.jl:59-67) -- run as
ONE batched launch over all waypoints (of one or many trajectories):

* ``IneqConst``  -> ``kin_ineq_const_batch`` (k_coll with truncation
  ``margin + 0.05`` and the ``- margin`` offset fused in);
* ``PoseConstraint`` -> ``kin_pose_const_batch`` (k_fk with rpy Jacobian +
  k_pose_residual).

The optimiser stays on the host, as the reference's does: ``Objective``,
``ConfigurationConstraint``, ``EqConst`` are small host-side assemblies and
``plan_trajectory`` drives SciPy's SLSQP (the reference's ``solver=:SCIPY``
path).  NLopt and Ipopt are not installed, so ``solver=:NLOPT`` / ``:IPOPT`` are
refused; ``solver="SLSQP_BOUNDED"`` (the default) is SciPy's SLSQP with the
joint-limit bounds the reference's NLopt path sets (src/planning.jl:364-369) --
SciPy's implementation, not NLopt's -- and reports its status as a symbol.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib as K
from .collision import SweptSphereCollisionChecker, UnionSDF
from .mechanism import Link, Mechanism, _device, _same_device

_DT = {torch.float32: K.KIN_F32, torch.float64: K.KIN_F64}


# ---------------------------------------------------------------------------- host side
class Objective:
    """src/planning.jl:1-28: xi^T A xi with A = kron(A_acc, diag(w^2)) (finite-difference acceleration)."""

    def __init__(self, n_wp: int, weights):
        from scipy import sparse
        w = np.asarray(weights, np.float64)
        A_sub = np.zeros((n_wp, n_wp))
        blk = np.array([[1, -2, 1], [-2, 4, -2], [1, -2, 1]], np.float64)
        for i in range(1, n_wp - 1):
            A_sub[i - 1:i + 2, i - 1:i + 2] += blk
        self.A = sparse.csc_matrix(np.kron(A_sub, np.diag(w ** 2)))
        self.n_dim = self.A.shape[1]

    def __call__(self, xi, grad: Optional[np.ndarray] = None) -> float:
        tmp = self.A @ np.asarray(xi, np.float64)
        if grad is not None and len(grad) > 0:
            grad[:] = 2.0 * tmp
        return float(np.dot(xi, tmp))


class IneqConst:
    """src/planning.jl:32-68.  ``__call__(xi, val_vec, jac_mat)`` fills the reference's dense
    layout (val_vec [n_coll*n_wp], jac_mat [n_dof*n_wp, n_coll*n_wp], block diagonal) from one
    GPU launch over the n_wp waypoints; ``eval_batch`` is the device-resident batched form."""

    def __init__(self, sscc: SweptSphereCollisionChecker, joints, sdf: UnionSDF, n_wp: int, margin: float,
                 dtype=torch.float64):
        self.sscc, self.joints, self.sdf = sscc, list(joints), sdf
        self.n_wp = int(n_wp)
        self.n_dof = len(self.joints) + (3 if sscc.mech.with_base else 0)
        self.n_coll = len(sscc.sphere_links)
        self.n_cons = self.n_coll * self.n_wp
        self.margin = float(margin)
        self.plan = sscc.plan(self.joints, dtype=dtype)
        self.dtype = dtype
        self.jac_mat = np.zeros((self.n_dof * self.n_wp, self.n_cons))
        self.val_vec = np.zeros(self.n_cons)

    def eval_batch(self, Q: torch.Tensor, with_jac=True, stream=None):
        """Q: device [n_dof, N] (any number of waypoints / trajectories side by side) ->
        vals [n_coll, N], jac [n_coll, n_dof, N] (or None).  Async on the stream."""
        if Q.dtype != self.dtype or not Q.is_cuda or Q.dim() != 2 or Q.shape[0] != self.n_dof or Q.stride(1) != 1:
            raise ValueError(f"Q must be a CUDA {self.dtype} tensor of shape ({self.n_dof}, N)")
        N = Q.shape[1]
        V = torch.empty((self.n_coll, N), dtype=self.dtype, device=Q.device)
        G = torch.empty((self.n_coll, self.n_dof, N), dtype=self.dtype, device=Q.device) if with_jac else None
        st = (stream or torch.cuda.current_stream(Q.device)).cuda_stream
        K.check(K.lib().kin_ineq_const_batch(self.plan._h, self.sdf._h, self.margin, Q.data_ptr(), Q.stride(0), N,
                                             V.data_ptr(), N, G.data_ptr() if G is not None else None, N, st))
        return V, G

    def __call__(self, xi, val_vec: np.ndarray, jac_mat: np.ndarray):
        xi = np.asarray(xi, np.float64)
        Q = torch.tensor(xi.reshape(self.n_wp, self.n_dof).T.copy(), dtype=self.dtype, device=_device())
        V, G = self.eval_batch(Q)
        v = V.double().cpu().numpy()    # [n_coll, n_wp]
        g = G.double().cpu().numpy()    # [n_coll, n_dof, n_wp]
        nd, nc = self.n_dof, self.n_coll
        for i in range(self.n_wp):
            jac_mat[nd * i:nd * (i + 1), nc * i:nc * (i + 1)] = g[:, :, i].T
        val_vec[:] = v.T.reshape(-1)


class PartialConstraint:
    idx_wp: int
    n_dof: int
    n_cons: int


class ConfigurationConstraint(PartialConstraint):
    """src/planning.jl:72-88: q(idx_wp) == q_const."""

    def __init__(self, idx_wp: int, n_dof: int, q_const):
        self.idx_wp, self.n_dof, self.n_cons = int(idx_wp), int(n_dof), int(n_dof)
        self.q_const = np.asarray(q_const, np.float64)

    def __call__(self, q, val_vec, jac_mat):
        j0 = (self.idx_wp - 1) * self.n_dof
        jac_mat[j0:j0 + self.n_dof, :] = -np.eye(self.n_dof)
        val_vec[:] = self.q_const - np.asarray(q, np.float64)


class PoseConstraint(PartialConstraint):
    """src/planning.jl:90-138: pose of each move link at waypoint idx_wp == target
    (position, plus rpy when with_rot); Jacobian = get_jacobian!(..., rpy_jac=true)."""

    def __init__(self, idx_wp: int, n_dof: int, move_links, target_poses, with_rots, mech: Mechanism, joints,
                 dtype=torch.float64):
        if isinstance(move_links, Link):
            move_links, target_poses, with_rots = [move_links], [target_poses], [with_rots]
        self.idx_wp, self.n_dof = int(idx_wp), int(n_dof)
        self.move_links, self.with_rots = list(move_links), [bool(w) for w in with_rots]
        self.target_poses = [np.asarray(T, np.float64).reshape(4, 4) for T in target_poses]
        self.n_cons = sum(6 if w else 3 for w in self.with_rots)
        self.mech, self.joints, self.dtype = mech, list(joints), dtype
        self.plans = [mech.plan(self.joints, out_links=[l], jac_link=l, jac_joints=self.joints, with_rot=w,
                                rpy_jac=w, dtype=dtype) for l, w in zip(self.move_links, self.with_rots)]

    def eval_batch(self, k: int, Q: torch.Tensor, targets: torch.Tensor, stream=None):
        """Move link k for N configurations: Q [n_dof, N], targets [12, N] (3x4 column-major) ->
        (vals [dim, N], jac [n_dof, dim, N], poses [12, N]) on the device."""
        p = self.plans[k]
        dim = 6 if self.with_rots[k] else 3
        N = Q.shape[1]
        if Q.dtype != self.dtype or not Q.is_cuda or Q.shape[0] != self.n_dof or Q.stride(1) != 1:
            raise ValueError(f"Q must be a CUDA {self.dtype} tensor of shape ({self.n_dof}, N)")
        if targets.dtype != self.dtype or targets.shape != (12, N) or targets.stride(1) != 1:
            raise ValueError("targets must be (12, N) in the plan dtype")
        _same_device(targets, Q, "targets")
        P = torch.empty((12, N), dtype=self.dtype, device=Q.device)
        V = torch.empty((dim, N), dtype=self.dtype, device=Q.device)
        J = torch.empty((self.n_dof, dim, N), dtype=self.dtype, device=Q.device)  # zero-filled plan
        st = (stream or torch.cuda.current_stream(Q.device)).cuda_stream
        K.check(K.lib().kin_pose_const_batch(p._h, targets.data_ptr(), targets.stride(0), Q.data_ptr(), Q.stride(0),
                                             N, P.data_ptr(), N, V.data_ptr(), N, J.data_ptr(), N, st))
        return V, J, P

    def __call__(self, q, val_vec, jac_mat):
        dev = _device()
        Q = torch.tensor(np.asarray(q, np.float64), dtype=self.dtype, device=dev).reshape(-1, 1).contiguous()
        j0 = (self.idx_wp - 1) * self.n_dof
        i0 = 0
        for k, (T, w) in enumerate(zip(self.target_poses, self.with_rots)):
            tg = torch.tensor(np.concatenate([T[:3, :3].T.reshape(-1), T[:3, 3]]), dtype=self.dtype,
                              device=dev).reshape(12, 1)
            V, J, _ = self.eval_batch(k, Q, tg)
            dim = 6 if w else 3
            val_vec[i0:i0 + dim] = V[:, 0].double().cpu().numpy()
            # get_jacobian!(..., transpose(jac)): jac_mat[j0 + d, i0 + r] = J[r, d]; irrelevant
            # columns are left untouched, as get_jacobian! leaves them
            Jh = J[:, :, 0].double().cpu().numpy()  # [n_dof, dim]
            rel = [self.mech.is_relevant(j, self.move_links[k]) for j in self.joints]
            rel += [True] * (self.n_dof - len(self.joints))
            for d in range(self.n_dof):
                if rel[d]:
                    jac_mat[j0 + d, i0:i0 + dim] = Jh[d]
            i0 += dim


class EqConst:
    """src/planning.jl:140-176: stacked partial constraints."""

    def __init__(self, n_wp: int, cons_arr: Sequence[PartialConstraint]):
        self.n_dof = cons_arr[0].n_dof
        assert all(c.n_dof == self.n_dof for c in cons_arr)
        self.n_wp, self.cons_arr = int(n_wp), list(cons_arr)
        self.n_cons = sum(c.n_cons for c in cons_arr)
        self.jac_mat = np.zeros((self.n_dof * self.n_wp, self.n_cons))
        self.val_vec = np.zeros(self.n_cons)

    def __call__(self, xi, val_vec, jac_mat):
        X = np.asarray(xi, np.float64).reshape(self.n_wp, self.n_dof)
        i0 = 0
        for c in self.cons_arr:
            c(X[c.idx_wp - 1], val_vec[i0:i0 + c.n_cons], jac_mat[:, i0:i0 + c.n_cons])
            i0 += c.n_cons


def create_straight_trajectory(q_start, q_goal, n_wp: int) -> np.ndarray:
    """src/planning.jl:304-308."""
    q_start, q_goal = np.asarray(q_start, np.float64), np.asarray(q_goal, np.float64)
    step = (q_goal - q_start) / (n_wp - 1)
    return np.concatenate([q_start + step * i for i in range(n_wp)])


def construct_problem(sscc, joints, sdf, q_start, q_goal, n_wp, n_dof, margin, partial_consts=()):
    """src/planning.jl:310-330."""
    eq = [ConfigurationConstraint(1, n_dof, q_start), ConfigurationConstraint(n_wp, n_dof, q_goal)]
    eq += list(partial_consts)
    return (Objective(n_wp, np.ones(n_dof)), IneqConst(sscc, joints, sdf, n_wp, margin), EqConst(n_wp, eq),
            n_dof * n_wp)


def plan_trajectory(sscc: SweptSphereCollisionChecker, joints, sdf: UnionSDF, q_start, q_goal, n_wp: int,
                    margin=2e-2, partial_consts=(), ftol_abs=1e-3, solver="SLSQP_BOUNDED", maxiter=200):
    """src/planning.jl:332-401 -> (q_seq [n_dof, n_wp], status).  Constraint evaluations on the GPU.

    ``solver``: "SLSQP_BOUNDED" (SciPy SLSQP + joint-limit bounds; status ``:SUCCESS`` /
    ``:MAXEVAL_REACHED`` / ``:FAILURE``) or "SCIPY" (the reference's :SCIPY path: no bounds, returns
    SciPy's result).  "NLOPT" and "IPOPT" raise: those libraries are not installed."""
    from scipy.optimize import minimize
    from .collision import compute_coll_dists

    solver = str(solver).lstrip(":").upper()
    if solver in ("NLOPT", "IPOPT"):
        raise ValueError(f"solver :{solver} needs a library that is not installed; use 'SLSQP_BOUNDED' "
                         "(SciPy SLSQP with the joint-limit bounds) or 'SCIPY'")
    if solver not in ("SLSQP_BOUNDED", "SCIPY"):
        raise ValueError(f"unknown solver {solver!r}")
    m = sscc.mech
    n_dof = len(joints) + (3 if m.with_base else 0)
    assert len(q_start) == n_dof and len(q_goal) == n_dof
    for q in (q_start, q_goal):
        m.set_joint_angles(joints, q)
        assert np.all(compute_coll_dists(sscc, joints, sdf) > 0.0), "start / goal in collision"
    xi0 = create_straight_trajectory(q_start, q_goal, n_wp)
    F, G, H, n_whole = construct_problem(sscc, joints, sdf, q_start, q_goal, n_wp, n_dof, margin, partial_consts)

    def cached(cons):  # one GPU evaluation per iterate serves both fun and jac
        last = {}

        def ev(x):
            key = x.tobytes()
            if last.get("key") != key:
                cons(x, cons.val_vec, cons.jac_mat)
                last.update(key=key, val=cons.val_vec.copy(), jac=cons.jac_mat.T.copy())
            return last
        return (lambda x: ev(x)["val"]), (lambda x: ev(x)["jac"])

    g_val, g_jac = cached(G)
    h_val, h_jac = cached(H)
    grad = np.zeros(n_whole)
    cons = [{"type": "ineq", "fun": g_val, "jac": g_jac}, {"type": "eq", "fun": h_val, "jac": h_jac}]
    bounds = None
    if solver == "SLSQP_BOUNDED":
        lo = [j.lower_limit for j in joints] + ([-np.inf] * 3 if m.with_base else [])
        hi = [j.upper_limit for j in joints] + ([np.inf] * 3 if m.with_base else [])
        bounds = list(zip(lo * n_wp, hi * n_wp))
    res = minimize(lambda x: F(x, grad), xi0, jac=lambda x: (F(x, grad), grad.copy())[1], method="SLSQP",
                   bounds=bounds, constraints=cons, options={"ftol": ftol_abs, "maxiter": maxiter})
    q_seq = res.x.reshape(n_wp, n_dof).T
    if solver == "SCIPY":
        return q_seq, res
    status = ":SUCCESS" if res.success else (":MAXEVAL_REACHED" if res.status == 9 else ":FAILURE")
    return q_seq, status


def collision_aware_ik(m: Mechanism, link: Link, joints, target_pose, sscc: SweptSphereCollisionChecker,
                       sdf: UnionSDF, use_bistage=True, ftol=1e-5, with_rot=True, max_iters=200, lam=1e-2,
                       max_step=0.5, margin=0.02, solver="DLS"):
    """``inverse_kinematics!(m, link, joints, target, sscc, sdf; use_bistage)`` (src/inverse_kinematics.jl:1-21);
    see ``kinhip.inverse_kinematics_``.  -> (q, status); sets the mechanism's angles.

    ``solver="DLS"`` (default): stage 1 (use_bistage) is the collision-free solve with the reference's
    ftol_abs rule (``_dls_ik_ftol``), stage 2 the batched collision-aware kernel
    (``CollisionIKPlan.ik_coll``, kin_ik_coll_batch: the reference's rpy objective plus the
    IneqConst(sscc, joints, sdf, 1, margin) sphere rows, 3 restarts: with use_bistage the first from the
    angles stage 1 started from (kin_ik_coll_batch_alt), the others seeded draws) on a batch of one, converged
    to |dp|, |d rpy| < 1e-6 with every sphere at >= margin - 1e-6 (status ``:FTOL_REACHED``).  When no
    attempt converges (a pose the constraint forbids) the kernel returns the attempt whose end state has
    the lowest merit |dp|^2 + |d rpy|^2 + max(0, margin - min d)^2 (the penalty problem's value; ties: the
    earlier attempt, so the stage-1-seeded attempt 0 wins over equal restarts), status
    ``:MAXEVAL_REACHED``.  ``ftol`` applies to stage 1 only: stage 2 is judged on the 1e-6 rule above.
    ``solver="SLSQP"``: stage 2 by SciPy's SLSQP on the host (the reference uses NLopt's LD_SLSQP), one
    GPU evaluation per iterate, ``ftol`` as the reference's ftol_abs."""
    from .collision import CollisionIKPlan
    from .mechanism import _dls_ik_ftol

    q_start = np.asarray(m.get_joint_angles(joints), np.float64)  # stage 2's restart attempt 1 starts here
    if use_bistage:  # stage 1: the collision-free problem seeds stage 2 (src/inverse_kinematics.jl:8-13)
        _dls_ik_ftol(m, link, joints, target_pose, ftol, with_rot, max_iters, lam, max_step)
    n_dof = len(joints) + (3 if m.with_base else 0)
    T = np.asarray(target_pose, np.float64).reshape(4, 4)
    dev = _device()
    tg = torch.tensor(np.concatenate([T[:3, :3].T.reshape(-1), T[:3, 3]]), dtype=torch.float64,
                      device=dev).reshape(12, 1)
    if str(solver).upper() == "DLS":
        plan = CollisionIKPlan(sscc, link, joints, dtype=torch.float64)
        Q0 = torch.tensor(m.get_joint_angles(joints), dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
        Q = torch.empty_like(Q0)
        Qa = torch.tensor(q_start, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous() if use_bistage else None
        Q, it, err = plan.ik_coll(sdf, tg.contiguous(), Q, Q0=Q0, margin=margin, with_rot=2 if with_rot else 0,
                                  max_iters=max_iters, restarts=3, lam=lam, max_step=max_step, tol_pos=1e-6,
                                  tol_rot=1e-6, Q_alt=Qa)
        q = Q[:, 0].cpu().numpy()
        m.set_joint_angles(joints, q)
        return q, (":FTOL_REACHED" if int(it[0]) <= max_iters else ":MAXEVAL_REACHED")
    if str(solver).upper() != "SLSQP":
        raise ValueError(f"unknown solver {solver!r} (DLS or SLSQP)")
    from scipy.optimize import minimize
    # objective: PoseConstraint's residual [p - p*; rpy - rpy*] and its rpy Jacobian on the GPU
    pc = PoseConstraint(1, n_dof, link, T, with_rot, m, joints, dtype=torch.float64)
    # src/inverse_kinematics.jl:16 (a checker without spheres has no constraints: the reference's own
    # PR2 test builds one, test/test_inverse_kinematics.jl:63, with an un-iterated generator)
    G = IneqConst(sscc, joints, sdf, 1, margin, dtype=torch.float64) if sscc.sphere_links else None
    rel = np.array([m.is_relevant(j, link) for j in joints] + [True] * (n_dof - len(joints)))

    def pose_eval(x):
        Q = torch.tensor(np.asarray(x, np.float64), dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
        V, J, _ = pc.eval_batch(0, Q, tg)
        v = V[:, 0].cpu().numpy()               # now - target
        Jh = J[:, :, 0].cpu().numpy() * rel[:, None]  # [n_dof, dim]
        return float(np.dot(v, v)), 2.0 * Jh @ v  # f = sum(diff.^2), grad = -2 J^T diff

    def cached(fn):
        last = {}

        def ev(x):
            k = np.asarray(x, np.float64).tobytes()
            if last.get("k") != k:
                last.update(k=k, r=fn(x))
            return last["r"]
        return ev

    fo = cached(pose_eval)

    def g_eval(x):
        G(x, G.val_vec, G.jac_mat)
        return G.val_vec + 1e-8, G.jac_mat.T.copy()  # nloptize(G) <= 1e-8  <=>  dist - margin >= -1e-8
    go = cached(g_eval)
    lo = [j.lower_limit for j in joints] + [-np.inf] * (n_dof - len(joints))
    hi = [j.upper_limit for j in joints] + [np.inf] * (n_dof - len(joints))
    x0 = np.clip(m.get_joint_angles(joints), lo, hi)
    cons = [{"type": "ineq", "fun": lambda x: go(x)[0], "jac": lambda x: go(x)[1]}] if G is not None else []
    res = minimize(lambda x: fo(x)[0], x0, jac=lambda x: fo(x)[1], method="SLSQP", bounds=list(zip(lo, hi)),
                   constraints=cons, options={"ftol": ftol, "maxiter": max_iters})  # ftol_abs, as the reference
    q = np.asarray(res.x, np.float64)
    m.set_joint_angles(joints, q)
    status = ":FTOL_REACHED" if res.success else (":MAXEVAL_REACHED" if res.status == 9 else ":FAILURE")
    return q, status
