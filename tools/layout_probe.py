"""Layout probe: FK + J fp32 (specialised) at 2^20 with the SoA rows ld = N (the
Julia shim's ROCMatrix(N, 8) / ROCArray(N, 6, 8)) or padded, q and outputs padded apart, warm (back-to-
back launches over the same buffers) and cold (each launch after a 1 GiB read of another buffer), and
at 2^22 (arrays 4x the Infinity Cache), to tell HBM channel aliasing from lost Infinity-Cache reuse.
    python tools/layout_probe.py"""
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
plan = m.plan(arm, out_links=[gl], jac_link=gl, jac_joints=arm, with_rot=True, dtype=torch.float32)
plan.specialize()
lo, hi = [j.lower_limit for j in arm], [j.upper_limit for j in arm]
scrub = torch.empty(1 << 28, dtype=torch.float32, device=dev)
st = torch.cuda.Stream(dev)


def bufs(N, padq, pado):
    Qb = torch.empty((8, N + padq), dtype=torch.float32, device=dev)
    Qb[:, :N] = kinhip.uniform_configs(lo, hi, N, dtype=torch.float32, device=dev)
    P = torch.zeros((1, 12, N + pado), dtype=torch.float32, device=dev)[:, :, :N]
    J = torch.zeros((8, 6, N + pado), dtype=torch.float32, device=dev)[:, :, :N]
    return Qb[:, :N], P, J


def warm(N, Q, P, J, k):
    with torch.cuda.stream(st):
        for _ in range(5):
            plan.run(Q, P, J, stream=st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(k):
            plan.run(Q, P, J, stream=st)
        e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k * 1e3


def cold(N, Q, P, J, k=10):
    ev = []
    with torch.cuda.stream(st):
        for _ in range(k):
            scrub.add_(1.0)  # reads and writes 1 GiB: evicts the 256 MiB Infinity Cache
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            plan.run(Q, P, J, stream=st)
            e1.record(st)
            ev.append((e0, e1))
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / k * 1e3


for lg in (20, 22):
    N = 1 << lg
    for padq, pado in ((0, 0), (256, 256), (0, 256), (256, 0), (64, 64), (2048, 2048)):
        if lg == 22 and (padq, pado) not in ((0, 0), (256, 256)):
            continue
        Q, P, J = bufs(N, padq, pado)
        w = warm(N, Q, P, J, 30 if lg == 20 else 10)
        c = cold(N, Q, P, J)
        print(f"N=2^{lg} padq={padq:5d} pado={pado:5d}: warm {w:7.2f} us ({272 * N / w / 1e3:6.0f} GB/s)  "
              f"cold {c:7.2f} us ({272 * N / c / 1e3:6.0f} GB/s)", flush=True)
        del Q, P, J
    # the headline's tiled layout
    Q = kinhip.tiled(kinhip.uniform_configs(lo, hi, N, dtype=torch.float32, device=dev), 8192)
    nt = Q.shape[0]
    P = torch.zeros((nt, 1, 12, 8192), dtype=torch.float32, device=dev)
    J = torch.zeros((nt, 8, 6, 8192), dtype=torch.float32, device=dev)

    def run_t():
        plan.run_tiled(Q, N, P, J, stream=st)

    with torch.cuda.stream(st):
        for _ in range(5):
            run_t()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            run_t()
        e1.record(st)
    torch.cuda.synchronize()
    w = e0.elapsed_time(e1) / 20 * 1e3
    ev = []
    with torch.cuda.stream(st):
        for _ in range(10):
            scrub.add_(1.0)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            run_t()
            b.record(st)
            ev.append((a, b))
    torch.cuda.synchronize()
    c = sum(a.elapsed_time(b) for a, b in ev) / 10 * 1e3
    print(f"N=2^{lg} tiled 8192:          warm {w:7.2f} us ({272 * N / w / 1e3:6.0f} GB/s)  "
          f"cold {c:7.2f} us ({272 * N / c / 1e3:6.0f} GB/s)", flush=True)
    del Q, P, J

# the same bytes with no arithmetic (libkinprobe.so, the kernels' addressing): is the ld = N penalty the
# pattern's own?
import ctypes as C  # noqa: E402
PR = C.CDLL(os.path.join(ROOT, "kinematics.jl_amd", "lib", "libkinprobe.so"))
PR.kinprobe_pattern2.argtypes = [C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_void_p,
                                 C.c_void_p]
for lg in (20, 22):
    N = 1 << lg
    for pad in (0, 256):
        q = torch.zeros(8 * (N + pad), dtype=torch.float32, device=dev)
        o = torch.zeros(60 * (N + pad), dtype=torch.float32, device=dev)

        def go():
            assert PR.kinprobe_pattern2(8, 60, N, 0, N + pad, 1, q.data_ptr(), o.data_ptr(), st.cuda_stream) == 0
        for _ in range(5):
            go()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            go()
        e1.record(st)
        torch.cuda.synchronize()
        w = e0.elapsed_time(e1) / 20 * 1e3
        print(f"pattern N=2^{lg} pad={pad}: warm {w:7.2f} us ({272 * N / w / 1e3:6.0f} GB/s)", flush=True)
        del q, o
