"""Row padding of the plain-SoA collision legs (config 5, specialised kernels, 2^20 samples fp32): the
distances + gradients kernel and its access-pattern probe (8 rows in, 126 out) at ld = n + pad, and
the min-distance kernel; results must equal the unpadded run bit for bit.
    python tools/coll_pad_ab.py"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
sdf = kinhip.fridge_sdf(fr)
sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
dt = torch.float32
cp = sscc.plan(arm, dtype=dt).specialize()
n = 1 << 20
Q0 = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=555, dtype=dt,
                            device=dev)
P = C.CDLL(os.path.join(ROOT, "kinematics.jl_amd", "lib", "libkinprobe.so"))
P.kinprobe_pattern2.argtypes = [C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_void_p,
                                  C.c_void_p]
st = torch.cuda.current_stream(dev)


def timed(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


ref = None
for rep in range(2):
    for pad in (0, 64, 128, 256, 512, 1024, 4096):
        ld = n + pad
        Qb = torch.empty((8, ld), dtype=dt, device=dev)
        Qb[:, :n] = Q0
        Q = Qb[:, :n]
        D = torch.zeros((cp.n_sph, ld), dtype=dt, device=dev)[:, :n]
        G = torch.zeros((cp.n_sph, 8, ld), dtype=dt, device=dev)[:, :, :n]
        t_g = timed(lambda: cp.run(sdf, Q, dists=D, grads=G))
        t_m = timed(lambda: cp.run(sdf, Q, dists=False, min_dist=True))
        if ref is None:
            ref = (D.clone(), G.clone())
        same = torch.equal(D, ref[0]) and torch.equal(G, ref[1])
        pq = torch.zeros(8 * ld, dtype=dt, device=dev)
        po = torch.zeros(126 * ld, dtype=dt, device=dev)
        t_p = timed(lambda: P.kinprobe_pattern2(8, 126, n, 0, ld, 1, pq.data_ptr(), po.data_ptr(), st.cuda_stream))
        print(f"rep {rep} pad {pad:5d}: dists+grads {t_g:6.1f} us  pattern {t_p:6.1f} us  frac_of_pattern "
              f"{t_p / t_g:.3f}  min_dist {t_m:5.1f} us  identical {same}", flush=True)
        del Qb, Q, D, G, pq, po
