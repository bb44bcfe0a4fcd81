"""Config-4 IK: is the bench's batch loop bound by the host's submission rate?  Times 200 back-to-back
kin_ik_dls_batch_from calls (bench._ik_leg's loop) two ways: the host time to submit them (no synchronize)
and the total (synchronized), plus the ctypes call alone with preallocated outputs.
    python tools/ik_host_probe.py"""
import ctypes as C
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from kinhip import _lib as K  # noqa: E402
from kinhip import dist as D  # noqa: E402
import kinhip  # noqa: E402

ctx = D.init_from_env()
dev = ctx.device
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
gl = m.find_link("gripper_link")
plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=torch.float32)
bench._specialize(plan, kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
tgt, kw = bench.ik_shard(m, arm, gl, ctx, 65536, torch.float32)
N = tgt.shape[1]
Q0 = torch.zeros((8, N), dtype=torch.float32, device=dev)
stream = torch.cuda.Stream(dev)
R = 200
with torch.cuda.stream(stream):
    for _ in range(5):
        plan.ik_dls(tgt, torch.empty_like(Q0), stream=stream, Q0=Q0, **kw)
torch.cuda.synchronize()
for rep in range(2):
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for _ in range(R):
            plan.ik_dls(tgt, torch.empty_like(Q0), stream=stream, Q0=Q0, **kw)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"python loop: submit {(t1 - t0) / R * 1e6:.1f} us/call, total {(t2 - t0) / R * 1e6:.1f} us/call", flush=True)
    # the C-ABI call alone, outputs preallocated (what a Julia ccall loop costs)
    Q = torch.empty_like(Q0)
    it = torch.empty(N, dtype=torch.int32, device=dev)
    err = torch.empty((2, N), dtype=torch.float32, device=dev)
    prm = K.IkParams(64, float(kw.get("lam", 1e-2)), 1e-3, 1e-3, float(kw.get("max_step", 0.5)), int(kw.get("with_rot", 1)),
                     int(kw.get("restarts", 3)), int(kw.get("seed", 0)), 0, int(kw.get("index_base", 0)), 0.0)
    f = K.lib().kin_ik_dls_batch_from
    args = (plan._h, C.byref(prm), tgt.data_ptr(), N, Q0.data_ptr(), Q.data_ptr(), N, N, it.data_ptr(), err.data_ptr(),
            N, stream.cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(R):
        f(*args)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"ctypes only: submit {(t1 - t0) / R * 1e6:.1f} us/call, total {(t2 - t0) / R * 1e6:.1f} us/call", flush=True)
print("kw", kw)
