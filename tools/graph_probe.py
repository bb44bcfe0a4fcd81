"""Launch-gap probe: K plain launches of the FK+J step vs one HIP graph holding the step replayed K times
(torch.cuda.CUDAGraph around kin_plan_run, which is capture-safe)."""
import os
import sys
import time
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
gl = m.find_link("gripper_link")
plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32)
N, pad = 1 << 20, 256
lo, hi = [j.lower_limit for j in arm], [j.upper_limit for j in arm]
Qb = torch.empty((8, N + pad), dtype=torch.float32, device=dev)
Qb[:, :N] = kinhip.uniform_configs(lo, hi, N, dtype=torch.float32, device=dev)
Q = Qb[:, :N]
P = torch.empty((1, 12, N + pad), dtype=torch.float32, device=dev)[:, :, :N]
J = torch.empty((8, 6, N + pad), dtype=torch.float32, device=dev)[:, :, :N]
s = torch.cuda.Stream(dev)
K = 50


def timed(fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K, (time.perf_counter() - t0) * 1e6 / K


with torch.cuda.stream(s):
    for _ in range(10):
        plan.run(Q, P, J, stream=s)
for rep in range(3):
    with torch.cuda.stream(s):
        ev, wall = timed(lambda: [plan.run(Q, P, J, stream=s) for _ in range(K)])
    print(f"plain launches : {ev:6.2f} us/step (events) {wall:6.2f} us/step (wall)")
g1 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g1, stream=s):
    plan.run(Q, P, J, stream=s)
gK = torch.cuda.CUDAGraph()
with torch.cuda.graph(gK, stream=s):
    for _ in range(K):
        plan.run(Q, P, J, stream=s)
for rep in range(3):
    with torch.cuda.stream(s):
        ev, wall = timed(lambda: [g1.replay() for _ in range(K)])
    print(f"graph of 1 step x {K} replays: {ev:6.2f} us/step (events) {wall:6.2f} us/step (wall)")
    with torch.cuda.stream(s):
        ev, wall = timed(lambda: gK.replay())
    print(f"graph of {K} steps x 1 replay: {ev:6.2f} us/step (events) {wall:6.2f} us/step (wall)")
