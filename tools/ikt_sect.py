"""Section stamps of the collision-aware IK (k_ik_tree) on the bench's f3 stage 2: 4,096 fridge
targets per launch, fp32, specialised (S = 16 sphere lanes x G = 4 attempt groups), stage 2 from stage 1's
answers.  Run with the A/B build and KINHIP_JIT_DEFS=-DKINHIP_IKT_SECT=<k> (tools/gpu_session.sh ikt-sections):
prints, for the target whose write comes last (the batch's latency), its iterations and the cycles of section
k, and the same section's mean over all targets.
    KINHIP_LIB=.../libkinhip_ab.so KINHIP_JIT_DEFS=-DKINHIP_IKT_SECT=3 python tools/ikt_sect.py"""
import os
import re
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
sys.path.insert(0, ROOT)
import kinhip  # noqa: E402
from bench import fridge_scene  # noqa: E402

NAMES = {1: "tree walk", 2: "sphere sdf + rows", 3: "rows -> normal eq", 4: "pose error + checks", 5: "pose rows",
         6: "factor + solves", 7: "step + loop top"}
k = int(re.search(r"KINHIP_IKT_SECT=(\d)", os.environ.get("KINHIP_JIT_DEFS", "=0")).group(1) or 0)
dev = torch.device("cuda", 0)
dt = torch.float32
m, arm, sscc, sdf = fridge_scene()
gl = m.find_link("gripper_link")
nt = 4096
rng = np.random.default_rng(17)
tg = np.zeros((12, nt))
for i in range(nt):
    x, y, z, yaw = rng.uniform(0.9, 1.05), rng.uniform(-0.12, 0.12), rng.uniform(1.15, 1.32), rng.uniform(-0.3, 0.3)
    c, s_ = np.cos(yaw), np.sin(yaw)
    tg[:, i] = np.concatenate([np.array([[c, -s_, 0.0], [s_, c, 0.0], [0.0, 0.0, 1.0]]).T.reshape(-1), [x, y, z]])
tg = torch.tensor(tg, dtype=dt, device=dev).contiguous()
cplan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=dt).specialize()
kw = dict(max_iters=128, restarts=3, seed=1, with_rot=2)
Q0 = torch.zeros((8, nt), dtype=dt, device=dev)
Q1 = torch.empty_like(Q0)
cplan.ik_dls(tg, Q1, Q0=Q0, **kw)
for rep in range(3):
    Q2, it, err = cplan.ik_coll(sdf, tg, torch.empty_like(Q0), Q0=Q1, margin=0.02, **kw)
torch.cuda.synchronize()
e = err.double().cpu().numpy()
it = it.cpu().numpy()
last = int(np.argmax(e[1]))
print(f"section {k} ({NAMES.get(k, '-')}): slowest target {last} iters {it[last]} total {e[1][last]:.0f} cycles, "
      f"section {e[0][last]:.0f} cycles ({e[0][last] / max(e[1][last], 1):.3f}); mean over targets {e[0].mean():.0f} "
      f"of {e[1].mean():.0f}", flush=True)
