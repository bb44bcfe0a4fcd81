"""Where the fp32 DLS step's error against fp64 comes from (one step from q = 0, Fetch, the 4,096 targets of
tests/test_gpu_ik_fp32_bound.py): J rounded to fp32 vs the 6x6 damped solve done in fp32.  CPU only (numpy +
oracle).   python tools/ik_fp32_solve_error.py"""
import sys, numpy as np
sys.path.insert(0,'oracle'); sys.path.insert(0,'tests'); sys.path.insert(0,'kinematics.jl_amd')
import oracle as O
from conftest import ARM, golden
t = O.parse_urdf_tree(golden("fetch.urdf")); om = O.OracleMech(t)
ids = [t.joint_id(n) for n in ARM]; gl = t.link_id("gripper_link")
lo = np.nan_to_num(np.array([t.joint_lower[i-1] for i in ids]), neginf=-np.pi)
hi = np.nan_to_num(np.array([t.joint_upper[i-1] for i in ids]), posinf=np.pi)
rng = np.random.default_rng(11); N=4096
tgt = om.fk_batch(lo[:, None] + (hi - lo)[:, None] * rng.random((8, N)), ids, [gl])[0]
pose, J = om.fk_jac_batch(np.zeros((8,1)), ids, gl, ids)
J = J[:, :, 0].T  # 6x8
T0 = np.eye(4); T0[:3,:4] = pose[:,0].reshape(4,3).T
lam2 = 1e-4
E = np.zeros((6, N))
for k in range(N):
    Tt = np.eye(4); Tt[:3,:4] = tgt[:,k].reshape(4,3).T
    E[:3,k] = Tt[:3,3]-T0[:3,3]; E[3:,k] = O.rot_error(Tt, T0)
def dls(J, E, dt=np.float64):
    J = J.astype(dt); A = J@J.T + dt(lam2)*np.eye(6, dtype=dt)
    L = np.linalg.cholesky(A.astype(dt)).astype(dt)
    y = np.linalg.solve(L.astype(dt), E.astype(dt)); y = np.linalg.solve(L.T, y)
    return (J.T@y).astype(np.float64)
d64 = dls(J, E)
# (a) J rounded to fp32 / perturbed by 1e-7 relative, exact solve
Ja = J.astype(np.float32).astype(np.float64)
da = dls(Ja, E)
Jb = J*(1+ rng.normal(size=J.shape)*2e-7)
db = dls(Jb, E)
# (b) exact J, fp32 normal equations + solve
dc = dls(J, E, np.float32)
# (c) fp32 solve + one refinement step in fp32
def dls_ref(J, E):
    J32=J.astype(np.float32); A=(J32@J32.T + np.float32(lam2)*np.eye(6,dtype=np.float32))
    L=np.linalg.cholesky(A); y=np.linalg.solve(L.T, np.linalg.solve(L, E.astype(np.float32)))
    r = E.astype(np.float32) - A@y
    y = y + np.linalg.solve(L.T, np.linalg.solve(L, r))
    return (J32.T@y).astype(np.float64)
dd = dls_ref(J, E)
for name, d in (("J fp32-rounded", da), ("J 2e-7 noise", db), ("fp32 solve", dc), ("fp32 solve+refine", dd)):
    dev = np.abs(d - d64)
    # the kernel also clamps the step to max_step 0.5 in inf norm: scale
    print(f"{name:20s} max {dev.max():.2e}  p50 {np.median(dev.max(0)):.2e}")
print("sv of J(0):", np.linalg.svd(J, compute_uv=False))
