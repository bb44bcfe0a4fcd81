"""Door-sweep A/B (bench.py's f2 leg, specialised fp32): `blocks` timed blocks of 20 launches each,
printing the median and minimum per-launch time and a checksum of the outputs (identical results across
library builds show as equal checksums).  KINHIP_LIB selects the library.   python tools/scene_ab.py [blocks]"""
import os
import statistics
import sys
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))
import kinhip  # noqa: E402

dev = torch.device("cuda", 0)
m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
arm = [m.find_joint(n) for n in kinhip.FETCH_ARM_JOINTS]
dt = torch.float32
cp = sscc.plan(arm, dtype=dt).specialize()
n = 1 << 20
Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, seed=556, dtype=dt,
                           device=dev)
asdf = kinhip.AttachedUnionSDF(fr, [fr.find_joint("door_joint")])
if os.environ.get("SCENE_AB_CONST") == "1":  # kin_plan_specialize_scene: the fridge's tables compiled in too
    cp.specialize_scene(asdf)
g = torch.Generator().manual_seed(90)
SQ = torch.zeros((4, n), dtype=torch.float64)
SQ[0] = torch.rand(n, generator=g, dtype=torch.float64) * 2.4
SQ[1] = 1.2
SQ = SQ.to(dt).to(dev).contiguous()
blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 15
if os.environ.get("SCENE_AB_FRESH") == "1":  # (round 4's form: contiguous rows, outputs allocated per call)
    run = lambda: cp.run(asdf, Q, grads=True, min_dist=True, scene_q=SQ)  # noqa: E731
else:  # the bench leg's form: rows padded to n + 256, preallocated outputs
    ld = n + 256
    Qb = torch.empty((8, ld), dtype=dt, device=dev)
    Qb[:, :n] = Q
    SQb = torch.empty((4, ld), dtype=dt, device=dev)
    SQb[:, :n] = SQ
    Dp = torch.zeros((cp.n_sph, ld), dtype=dt, device=dev)[:, :n]
    Gp = torch.zeros((cp.n_sph, 8, ld), dtype=dt, device=dev)[:, :, :n]
    run = lambda: cp.run(asdf, Qb[:, :n], dists=Dp, grads=Gp, min_dist=True, scene_q=SQb[:, :n])  # noqa: E731
# SCENE_AB_STREAM=1: launches on a created stream (the bench's _timed_calls form) instead of the null stream
st = torch.cuda.Stream() if os.environ.get("SCENE_AB_STREAM") == "1" else torch.cuda.current_stream()
with torch.cuda.stream(st):
    for _ in range(5):
        r = run()
torch.cuda.synchronize()
ts = []
for _ in range(blocks):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record(st)
        for _ in range(20):
            r = run()
        e1.record(st)
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 20 * 1e3)
chk = (float(r[0].double().abs().sum()), float(r[1].double().abs().sum()), float(r[2].double().sum()))
print(f"{'const' if os.environ.get('SCENE_AB_CONST') == '1' else 'data '} scene median {statistics.median(ts):6.1f}us min {min(ts):6.1f}us max {max(ts):6.1f}us first {ts[0]:6.1f}us "
      f"chk {chk[0]:.9e} {chk[1]:.9e} {chk[2]:.9e}", flush=True)
