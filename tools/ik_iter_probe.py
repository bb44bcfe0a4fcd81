"""Per-iteration cost of the specialised fp32 IK kernel at 1, 2, 4 waves per SIMD: tol 0 (no target
converges), no restarts, max_iters 8 and 16 -> (t16 - t8) / 8 per iteration (the first 16 iterations:
angles stay near their seeds, as in a real solve; longer runs drift the continuous joints into the
library sincos path).
    python tools/ik_iter_probe.py"""
import os
import sys
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
gl = m.find_link("gripper_link")
dt = torch.float64 if os.environ.get("AB_F64") else torch.float32
NS = [int(x) for x in os.environ.get("IK_NS", "65536,131072,262144").split(",")]
plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt).specialize()
rot = int(os.environ.get("AB_ROT", "1"))
for n in NS:
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=4242, dtype=dt,
                                device=dev)
    tgt = plan.run(Qt)[0][0].contiguous()
    Q0 = torch.zeros((8, n), dtype=dt, device=dev)
    res = {}
    for it in (8, 16):
        kw = dict(max_iters=it, restarts=0, seed=0, lam=1e-2, max_step=0.5, tol_pos=0.0, tol_rot=0.0, with_rot=rot)
        Q = Q0.clone()
        plan.ik_dls(tgt, Q, Q0=Q0, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            plan.ik_dls(tgt, Q, Q0=Q0, **kw)
        e1.record()
        torch.cuda.synchronize()
        res[it] = e0.elapsed_time(e1) / 10 * 1e3
    per = (res[16] - res[8]) / 8
    print(f"{str(dt)[6:]} rot={rot} n={n} ({n // 65536} waves/SIMD): t8 {res[8]:.1f} us t16 {res[16]:.1f} us -> "
          f"{per:.3f} us/iteration ({per * 1e3 / (n // 65536):.0f} ns per wave-iteration)", flush=True)
if os.environ.get("AB_G4"):
    # the phase-2 kernel shape: 4 lanes per target (attempts 0-3 side by side), one wave per SIMD
    n = 16384
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=4242, dtype=dt,
                                device=dev)
    tgt = plan.run(Qt)[0][0].contiguous()
    Q0 = torch.zeros((8, n), dtype=dt, device=dev)
    res = {}
    for mi in (32, 64):
        kw = dict(max_iters=mi, restarts=3, seed=0, lam=1e-2, max_step=0.5, tol_pos=0.0, tol_rot=0.0, with_rot=rot,
                  lanes=4)
        Q = Q0.clone()
        plan.ik_dls(tgt, Q, Q0=Q0, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            plan.ik_dls(tgt, Q, Q0=Q0, **kw)
        e1.record()
        torch.cuda.synchronize()
        res[mi] = e0.elapsed_time(e1) / 10 * 1e3
    print(f"G=4 (lanes=4), {n} targets = 1 wave per SIMD: attempts of 8 / 16 iterations {res[32]:.1f} / {res[64]:.1f} us"
          f" -> {(res[64] - res[32]) / 8:.3f} us/iteration", flush=True)
