"""Per-section cycles of one IK iteration (diagnostic A/B build: KINHIP_IK_SECT stamps, see
kinhip_ik_dev.h), specialised kernel, 65,536 targets (one wave per SIMD), tol 0, no restarts.
    KINHIP_LIB=.../libkinhip_ab.so KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=<k> python tools/ik_sect.py"""
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
plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt).specialize()
n = int(os.environ.get("IK_N", 65536))
iters = 32
Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=4242, dtype=dt,
                            device=dev)
tgt = plan.run(Qt)[0][0].contiguous()
Q0 = torch.zeros((8, n), dtype=dt, device=dev)
kw = dict(max_iters=iters, restarts=0, seed=0, lam=1e-2, max_step=0.5, tol_pos=0.0, tol_rot=0.0,
          with_rot=int(os.environ.get("AB_ROT", "1")))
Q = Q0.clone()
for _ in range(3):
    _, it, err = plan.ik_dls(tgt, Q, Q0=Q0, **kw)
torch.cuda.synchronize()
e = err.double()
k = os.environ.get("KINHIP_JIT_DEFS", "")
print(f"{k}: section {e[0].mean().item() / (iters + 1):.0f} cycles/iteration, lane total "
      f"{e[1].mean().item() / (iters + 1):.0f} cycles/iteration (n={n}, {str(dt)[6:]})", flush=True)
