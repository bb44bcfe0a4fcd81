"""When does the fp32 DLS IK need its fp64 damped solve?  Along config-4 trajectories
(attempt 0 from q0 = 0, 4,096 Fetch targets from the bench's within-limit distribution), per iteration:
the fp32 normal equations' error against fp64 (the same fp32-rounded J; numpy float32 emulation of the
kernel's fp32 solve) against a cheap lower bound of lambda_min(J J^T + lambda^2 I) from the fp32 Cholesky
factor, 1 / |L^-1|_F^2.  CPU only.   python tools/ik_cond_explore.py"""
import sys
import numpy as np
sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'kinematics.jl_amd')
import oracle as O
from conftest import ARM, golden

t = O.parse_urdf_tree(golden("fetch.urdf")); om = O.OracleMech(t)
ids = [t.joint_id(n) for n in ARM]; gl = t.link_id("gripper_link")
lo = np.nan_to_num(np.array([t.joint_lower[i - 1] for i in ids]), neginf=-np.pi)
hi = np.nan_to_num(np.array([t.joint_upper[i - 1] for i in ids]), posinf=np.pi)
rng = np.random.default_rng(4242); N = 4096
tgt = om.fk_batch(lo[:, None] + (hi - lo)[:, None] * rng.random((8, N)), ids, [gl])[0]
lam2 = 1e-4


def chol32(A):  # A [N,6,6] float32 -> L, pivots (the kernel's inverse-diagonal form, in float32)
    n = A.shape[1]; L = np.zeros_like(A); ip = np.zeros(A.shape[:2], np.float32); piv = np.zeros_like(ip)
    for j in range(n):
        d = A[:, j, j] - np.einsum('nk,nk->n', L[:, j, :j], L[:, j, :j]).astype(np.float32)
        piv[:, j] = d; ip[:, j] = 1 / np.sqrt(np.maximum(d, 1e-30)); L[:, j, j] = 1 / ip[:, j]
        for r in range(j + 1, n):
            L[:, r, j] = (A[:, r, j] - np.einsum('nk,nk->n', L[:, r, :j], L[:, j, :j]).astype(np.float32)) * ip[:, j]
    return L, piv


rows = []
for k in range(16):
    q, _, _ = om.ik_dls_batch(np.zeros((8, N)), ids, gl, tgt, max_iters=k, lam=1e-2, tol_pos=0.0, tol_rot=0.0,
                              max_step=0.5, restarts=0, seed=0)
    pose, J = om.fk_jac_batch(q, ids, gl, ids)  # J [8, 6, N]
    Jt = np.transpose(J, (2, 1, 0)).astype(np.float32)  # [N, 6, 8], fp32-rounded J (the kernel's)
    E = np.zeros((N, 6))
    for i in range(N):
        Tt = np.eye(4); Tt[:3, :4] = tgt[:, i].reshape(4, 3).T
        Tn = np.eye(4); Tn[:3, :4] = pose[:, i].reshape(4, 3).T
        E[i, :3] = Tt[:3, 3] - Tn[:3, 3]; E[i, 3:] = O.rot_error(Tt, Tn)
    J64 = Jt.astype(np.float64)
    A64 = J64 @ np.transpose(J64, (0, 2, 1)) + lam2 * np.eye(6)
    dq64 = np.einsum('nrc,nr->nc', J64, np.linalg.solve(A64, E[..., None])[..., 0])
    A32 = (Jt @ np.transpose(Jt, (0, 2, 1))).astype(np.float32) + np.float32(lam2) * np.eye(6, dtype=np.float32)
    L, piv = chol32(A32)
    y = np.linalg.solve(L.astype(np.float64), E[..., None]); y = np.linalg.solve(np.transpose(L, (0, 2, 1)).astype(np.float64), y)
    dq32 = np.einsum('nrc,nr->nc', J64, y[..., 0].astype(np.float32).astype(np.float64))
    Li = np.linalg.inv(L.astype(np.float64))
    lb = 1.0 / np.sum(Li * Li, axis=(1, 2))  # lower bound of lambda_min(A)
    sc = np.minimum(1.0, 0.5 / np.maximum(np.abs(dq64).max(1), 1e-30))  # the max_step clamp
    err = np.abs(dq32 - dq64).max(1) * sc
    rows.append((k, lb, err, piv.min(1)))
    ok = err <= 1e-5
    for tau in (1e-3, 3e-3, 1e-2):
        p = lb >= tau
        wave = p.reshape(-1, 64).all(1).mean()
        print(f"it {k:2d} tau {tau:.0e}: pass {p.mean():.3f} (waves all-pass {wave:.3f}); max err when pass "
              f"{err[p].max() if p.any() else 0:.1e}, when fail {err[~p].max() if (~p).any() else 0:.1e}; "
              f"err>1e-5 {(~ok).mean():.3f}")
