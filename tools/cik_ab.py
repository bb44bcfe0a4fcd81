"""Collision-aware IK A/B (tools/ab.py workload `cik`): the bench's f2/f3 legs (bench._scene_and_coll_ik_legs:
door sweep, f3 fridge, f3 attached-scene door, PR2 two arms + base, pillar scenes), specialised fp32, on the
library KINHIP_LIB names; one line of stage-2 times, the door sweep and the convergence fractions (equal
fractions across builds = the same answers; the parity tests pin the bits).   python tools/cik_ab.py [n]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kinhip import dist as D  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
ctx = D.init_from_env()
stream = torch.cuda.Stream(ctx.device)
o = bench._scene_and_coll_ik_legs(ctx, stream, n, 20)
f3, sd, pr = o["f3_collision_ik"], o["f3_collision_ik_scene_door"], o["f3_pr2_collision_ik"]
p4, p64 = o["f3_collision_ik_pillar_4096"], o["f3_collision_ik_pillar_65536"]
print(f"door {o['f2_scene_door_sweep']['avg_launch_us']:.1f}us | stage2 ms: f3 {f3['ms_stage2']:.4f} "
      f"scene {sd['ms_stage2']:.4f} pr2 {pr['ms_stage2']:.4f} | bistage ms: pillar4k {p4['ms_per_batch']:.4f} "
      f"pillar64k {p64['ms_per_batch']:.4f} | conv {f3['converged']:.6f} {sd['converged']:.6f} {pr['converged']:.6f}",
      flush=True)
