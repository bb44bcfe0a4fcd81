"""Generates tests/golden/fetch_fk_jac_golden.npz (committed).

1,024 seeded Fetch configurations, uniform within the URDF joint limits
(continuous joints U[-pi, pi]), of the 8 arm joints used by the reference's
tests (test/test_inverse_kinematics.jl:5-13).  Stored per configuration:
  q            (8, N)            joint angles
  poses        (25, 12, N)       world pose of every link (3x4 column-major)
  jac_geo      (8, 6, N)         get_jacobian(gripper_link, arm, with_rot=true)
  jac_rpy      (8, 6, N)         ... rpy_jac=true
  qb, jac_base (11, ...)         with_base variant (base x, y, theta appended)
produced by the C oracle (oracle/kin_oracle.c, a restatement of
src/algorithm.jl) and accepted only if the independent numpy formulation
(oracle/numpy_ref.py) agrees to 1e-12.

Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import numpy_ref as R  # noqa: E402
import oracle as O  # noqa: E402

ARM = ["torso_lift_joint", "shoulder_pan_joint", "shoulder_lift_joint", "upperarm_roll_joint",
       "elbow_flex_joint", "forearm_roll_joint", "wrist_flex_joint", "wrist_roll_joint"]


def main():
    tree = O.parse_urdf_tree(os.path.join(HERE, "fetch.urdf"))
    ids = [tree.joint_id(n) for n in ARM]
    N = 1024
    rng = np.random.default_rng(20261015)
    lo = np.array([tree.joint_lower[i - 1] for i in ids])
    hi = np.array([tree.joint_upper[i - 1] for i in ids])
    lo = np.where(np.isfinite(lo), lo, -np.pi)
    hi = np.where(np.isfinite(hi), hi, np.pi)
    q = lo[:, None] + (hi - lo)[:, None] * rng.random((8, N))
    m = O.OracleMech(tree)
    L = len(tree.link_names)
    poses = m.fk_batch(q, ids, list(range(1, L + 1)))
    gl = tree.link_id("gripper_link")
    _, jg = m.fk_jac_batch(q, ids, gl, ids, True, False)
    _, jr = m.fk_jac_batch(q, ids, gl, ids, True, True)
    qb = np.vstack([q, rng.uniform(-1, 1, (2, N)), rng.uniform(-np.pi, np.pi, (1, N))])
    mb = O.OracleMech(tree, with_base=True)
    pb, jb = mb.fk_jac_batch(qb, ids, gl, ids, True, False)

    # independent cross-check
    W = R.world_poses(tree, q, ids)
    err = max(np.abs(poses[l] - R.pose12(W[l])).max() for l in range(L))
    _, Jg = R.jacobian(tree, q, ids, gl, ids, True, False)
    _, Jr = R.jacobian(tree, q, ids, gl, ids, True, True)
    Tb, Jb = R.jacobian(tree, qb, ids, gl, ids, True, False, with_base=True)
    err = max(err, np.abs(jg - Jg.transpose(2, 1, 0)).max(), np.abs(pb - R.pose12(Tb)).max(),
              np.abs(jb - Jb.transpose(2, 1, 0)).max())
    # rpy rows: compare away from the pitch singularity
    ok = np.abs(np.cos(R.rpy_zyx(W[gl - 1][:, :3, :3])[:, 1])) > 1e-3
    err = max(err, np.abs((jr - Jr.transpose(2, 1, 0))[:, :, ok]).max())
    print("oracle vs numpy max abs diff:", err)
    assert err < 1e-12, err
    np.savez_compressed(os.path.join(HERE, "fetch_fk_jac_golden.npz"), joint_names=np.array(ARM), q=q,
                        poses=poses, jac_geo=jg, jac_rpy=jr, qb=qb, pose_base=pb, jac_base=jb)


if __name__ == "__main__":
    main()
