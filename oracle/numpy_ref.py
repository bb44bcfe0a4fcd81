"""Independent vectorised numpy formulation of batched FK + Jacobian (TEST INFRASTRUCTURE).

A second CPU statement of the same math as the C oracle, written differently
on purpose (Rodrigues rotations instead of quaternions, batch-vectorised root
-> leaf recursion over the parent chain instead of a cached leaf -> root stack)
so that golden vectors produced by the C oracle can be cross-checked by code
that shares no arithmetic with it.

Semantics followed: src/mechanism.jl:90-103 (joint_transform),
src/algorithm.jl:1-21 (world pose), :42-54 (pre-motion world joint axis),
:65-106 (geometric / rpy Jacobian columns, base columns), src/transform.jl:33-48.
"""
from __future__ import annotations

import numpy as np

FIXED, REVOLUTE, PRISMATIC = 0, 1, 2


def _rodrigues(axis, q):
    """[N,3,3] rotation by angle q[N] about unit-ish axis[3] (quaternion-equivalent)."""
    n = np.linalg.norm(axis)
    a = axis / n
    # Rotations.jl normalises (cos(q/2), axis*sin(q/2)): effective angle 2*atan2(n sin(q/2), cos(q/2))
    ang = 2.0 * np.arctan2(n * np.sin(0.5 * q), np.cos(0.5 * q))
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    s, c = np.sin(ang)[:, None, None], np.cos(ang)[:, None, None]
    return np.eye(3)[None] + s * K[None] + (1 - c) * (K @ K)[None]


def world_poses(tree, q, q_joint_ids, with_base=False, default_angles=None):
    """Returns [L, N, 4, 4] world transforms of every link (numpy, fp64)."""
    N = q.shape[1]
    L = len(tree.link_names)
    J = len(tree.joint_names)
    ang = np.zeros((J, N))
    if default_angles is not None:
        ang[:] = np.asarray(default_angles)[:, None]
    for c, jid in enumerate(q_joint_ids):
        ang[jid - 1] = q[c]
    root_T = np.tile(np.eye(4), (N, 1, 1))
    if with_base:
        x, y, th = q[len(q_joint_ids)], q[len(q_joint_ids) + 1], q[len(q_joint_ids) + 2]
        root_T[:, 0, 0] = np.cos(th); root_T[:, 0, 1] = -np.sin(th)
        root_T[:, 1, 0] = np.sin(th); root_T[:, 1, 1] = np.cos(th)
        root_T[:, 0, 3] = x; root_T[:, 1, 3] = y
    pj = np.full(L, -1)
    for j in range(J):
        pj[tree.joint_clink[j] - 1] = j
    out = np.zeros((L, N, 4, 4))
    done = np.zeros(L, bool)

    def rec(l):
        if done[l]:
            return out[l]
        j = pj[l]
        if j < 0:
            out[l] = root_T
        else:
            P = rec(tree.joint_plink[j] - 1)
            local = np.tile(tree.joint_pose[j], (N, 1, 1))
            t = tree.joint_type[j]
            if t == REVOLUTE:
                M = np.tile(np.eye(4), (N, 1, 1))
                M[:, :3, :3] = _rodrigues(tree.joint_axis[j], ang[j])
                local = local @ M
            elif t == PRISMATIC:
                M = np.tile(np.eye(4), (N, 1, 1))
                M[:, :3, 3] = tree.joint_axis[j][None] * ang[j][:, None]
                local = local @ M
            out[l] = P @ local
        done[l] = True
        return out[l]

    for l in range(L):
        rec(l)
    return out


def _subtree(tree, j):
    """links in the subtree of joint j's child (create_rptable, src/mechanism.jl:117-139)."""
    children = {}
    for k in range(len(tree.joint_names)):
        children.setdefault(tree.joint_plink[k], []).append(tree.joint_clink[k])
    s, stack = set(), [tree.joint_clink[j]]
    while stack:
        l = stack.pop()
        s.add(l)
        stack.extend(children.get(l, []))
    return s


def rpy_zyx(R):
    """[..., 3, 3] -> [..., 3] = [roll, pitch, yaw] (RotZYX extraction)."""
    t1 = np.arctan2(R[..., 1, 0], R[..., 0, 0])
    c1, s1 = np.cos(t1), np.sin(t1)
    t2 = np.arctan2(-R[..., 2, 0], R[..., 1, 0] * s1 + R[..., 0, 0] * c1)
    t3 = np.arctan2(R[..., 0, 2] * s1 - R[..., 1, 2] * c1, R[..., 1, 1] * c1 - R[..., 0, 1] * s1)
    return np.stack([t3, t2, t1], -1)


def jacobian(tree, q, q_joint_ids, link_id, jac_joint_ids, with_rot=True, rpy_jac=False, with_base=False):
    """-> pose [N,4,4], J [N, rows, ncol] (zero-filled, like get_jacobian)."""
    W = world_poses(tree, q, q_joint_ids, with_base)
    N = q.shape[1]
    T = W[link_id - 1]
    p = T[:, :3, 3]
    rows = 6 if with_rot else 3
    ncol = len(jac_joint_ids) + (3 if with_base else 0)
    Jm = np.zeros((N, rows, ncol))
    if rpy_jac:
        r = rpy_zyx(T[:, :3, :3])
        a2, a3 = -r[:, 1], -r[:, 2]
    for c, jid in enumerate(jac_joint_ids):
        j = jid - 1
        if link_id not in _subtree(tree, j):
            continue
        Fw = W[tree.joint_plink[j] - 1] @ tree.joint_pose[j][None]
        o = Fw[:, :3, 3]
        z = Fw[:, :3, :3] @ tree.joint_axis[j]
        if tree.joint_type[j] == REVOLUTE:
            Jm[:, :3, c] = np.cross(z, p - o)
            if with_rot:
                if rpy_jac:
                    x, y, zz = z[:, 0], z[:, 1], z[:, 2]
                    Jm[:, 3, c] = np.cos(a3) / np.cos(a2) * x - np.sin(a3) / np.cos(a2) * y
                    Jm[:, 4, c] = np.sin(a3) * x + np.cos(a3) * y
                    Jm[:, 5, c] = (-np.cos(a3) * np.sin(a2) / np.cos(a2) * x
                                   + np.sin(a3) * np.sin(a2) / np.cos(a2) * y + zz)
                else:
                    Jm[:, 3:, c] = z
        elif tree.joint_type[j] == PRISMATIC:
            Jm[:, :3, c] = z
        else:
            raise ValueError("fixed joint has no Jacobian column")
    if with_base:
        n = len(jac_joint_ids)
        bx, by = q[len(q_joint_ids)], q[len(q_joint_ids) + 1]
        Jm[:, 0, n] = 1
        Jm[:, 1, n + 1] = 1
        Jm[:, 0, n + 2] = -(p[:, 1] - by)
        Jm[:, 1, n + 2] = p[:, 0] - bx
        if with_rot:
            Jm[:, 5, n + 2] = 1
    return T, Jm


def pose12(T):
    """[N,4,4] -> [12, N] in the engine's 3x4 column-major SoA order."""
    return np.transpose(T[:, :3, :4], (2, 1, 0)).reshape(12, -1)
