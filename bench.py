"""Benchmark: Fetch FK + 6x8 geometric Jacobian evaluations per second (BASELINE.json metric).

Workload (BASELINE.json configs[2]): 2^20 Fetch arm configurations
per GPU, fp32, world pose of gripper_link (3x4) + 6x8 geometric Jacobian
(with_rot=true, rpy_jac=false, no base).  One step = one launch of the engine
over the whole batch; inputs are resident in HBM before timing starts.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 1048576]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Multi-GPU: configurations are independent, each rank evaluates its own 2^20
slice of one global counter-hashed dataset (weak scaling, no collective in the
timed region besides the bracketing barriers).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kinematics.jl_amd"))

import kinhip  # noqa: E402
from kinhip import dist as D  # noqa: E402

ARM = kinhip.FETCH_ARM_JOINTS
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
EXAMPLE_LINKS = ["l_gripper_finger_link", "r_gripper_finger_link", "wrist_flex_link", "wrist_roll_link",
                 "shoulder_lift_link", "upperarm_roll_link"]


def _time_plan(plan, Q, poses, jac, steps, warmup, ctx, stream):
    """K back-to-back launches bracketed by barrier + synchronize; HIP events on the launch stream."""
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            plan.run(Q, poses, jac, stream=stream)
    torch.cuda.synchronize()
    D.barrier(ctx)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        plan.run(Q, poses, jac, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    D.barrier(ctx)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dev_s = e0.elapsed_time(e1) / 1e3
    wall, dev_s = D.max_over_ranks(ctx, [wall, dev_s])
    return wall, dev_s


SPEC_ERRORS = []


def _specialize(plan, *kinds):
    """kin_plan_specialize; if run-time compilation fails the leg runs on the generic kernels and
    the failure is reported in the JSON line (`specialization_errors`) instead of aborting the bench."""
    try:
        plan.specialize(*kinds)
    except kinhip.KinError as e:  # noqa: PERF203
        SPEC_ERRORS.append(str(e)[:300])
    return plan


def _time_tiled(plan, Qt, n, poses, jac, steps, warmup, ctx, stream):
    """_time_plan for kin_plan_run_tiled."""
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            plan.run_tiled(Qt, n, poses, jac, stream=stream)
    torch.cuda.synchronize()
    D.barrier(ctx)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        plan.run_tiled(Qt, n, poses, jac, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    D.barrier(ctx)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dev_s = e0.elapsed_time(e1) / 1e3
    return D.max_over_ranks(ctx, [wall, dev_s])


# config 4's solver settings (fixed lambda, steps up to 0.5 rad).  The error-scaled damping lambda^2 + 0.01|e|^2
# with 1-rad steps solves 93% of the targets within 10 iterations of attempt 0 instead of 76% and raises
# success 0.995 -> 0.998 (tools/ik_damp_explore.py), but the two-phase schedule's length is set by the targets
# no attempt solves, and it measured slower (profiles/r04_ik_phase_traces.txt): reported as its own leg.
IK_KW = dict(max_iters=64, restarts=3, seed=0, lam=1e-2, max_step=0.5, damp_err=0.0, tol_pos=1e-3, tol_rot=1e-3)
IK_KW_DAMPED = dict(IK_KW, max_step=1.0, damp_err=0.01)


def ik_shard(m, arm, gl, ctx, n, dt):
    """Config 4's targets for this rank: FK of counter-hashed random q (reachable by construction) for
    global targets [rank * n, (rank + 1) * n), and the solver arguments.  `index_base` = the shard's
    global offset, so the restart draws -- and every result -- equal a single-process run's."""
    start, cnt = D.shard_range(n, ctx.rank)
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], cnt, start=start,
                                seed=4242, dtype=dt, device=ctx.device)
    # targets from a separate FK-only plan (generic kernel), so the headline kernel's rocprof
    # average covers the headline launches only
    tgt = m.plan(arm, out_links=[gl], dtype=dt).run(Qt)[0][0].contiguous()
    return tgt, dict(IK_KW, index_base=start)


def coll_shard(arm, ctx, n, dt, seed=555):
    """Config 5's samples for this rank: global configurations [rank * n, (rank + 1) * n)."""
    return kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, start=ctx.rank * n,
                                  seed=seed, dtype=dt, device=ctx.device)


def fridge_scene():
    """Config 5's scene: Fetch + 14 build-defined arm spheres, the fridge (door 2.0 rad, base (1.2, 0, 0))."""
    m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
    fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
    sdf = kinhip.fridge_sdf(fr)
    sscc = kinhip.add_fetch_arm_spheres(kinhip.SweptSphereCollisionChecker(m))
    return m, [m.find_joint(n_) for n_ in ARM], sscc, sdf


def _ik_leg(m, arm, gl, ctx, stream, n=65536, reps=100, spec=1, dt=torch.float32, over=None):
    """Config 4: batched DLS IK, `n` reachable targets per GPU (FK of seeded random q), q0 = 0,
    <= 64 iterations with 3 seeded restarts; success = converged to |dp| < 1e-3 and |rot| < 1e-3.
    Multi-GPU: the solutions (8 angles) and iteration counts are all-gathered to every rank over
    RCCL afterwards -- timed separately, not part of the solve rate.  `reps` back-to-back batches in the timed
    region (100: its fixed start and stop, ~70 us, were 5% of the 20 batches timed before round 6's last bench;
    tools/ik_host_probe.py: 66.3-67.4 us per batch over 200, host submission 10-15 us per call)."""
    plan = m.plan(arm, out_links=[gl], jac_link=gl, dtype=dt)
    if spec:
        _specialize(plan, kinhip.KIN_SPEC_FK | kinhip.KIN_SPEC_IK)
    tgt, kw = ik_shard(m, arm, gl, ctx, n, dt)
    kw.update(over or {})
    cnt = tgt.shape[1]
    Q0 = torch.zeros((8, cnt), dtype=dt, device=ctx.device)
    # every batch starts from Q0: read by the solver (kin_ik_dls_batch_from), the solutions go to a
    # fresh Q (written, not read) -- no copy of Q0 per batch
    with torch.cuda.stream(stream):
        plan.ik_dls(tgt, torch.empty_like(Q0), stream=stream, Q0=Q0, **kw)
    torch.cuda.synchronize()
    D.barrier(ctx)
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for _ in range(reps):
            Q, it, err = plan.ik_dls(tgt, torch.empty_like(Q0), stream=stream, Q0=Q0, **kw)
    torch.cuda.synchronize()
    D.barrier(ctx)
    wall = D.max_over_ranks(ctx, [time.perf_counter() - t0])[0]
    succ = (it <= 64).float().mean()  # kinhip.h: iters > max_iters <=> not converged
    out = {"value": n * ctx.world * reps / wall, "unit": "IK solves/s", "targets_per_gpu": n,
           "success_rate": float(succ), "ms_per_batch": wall / reps * 1e3,
           "dtype": "f32" if dt == torch.float32 else "f64",
           "params": (f"DLS lambda=1e-2{' + %g |e|^2' % kw['damp_err'] if kw.get('damp_err') else ''}, "
                      f"max_step={kw['max_step']}, 64 iters incl. 3 seeded restarts, q0=0, "
                      f"{['position', 'axis-angle', 'rpy (reference objective)'][int(kw.get('with_rot', 1))]} residual"),
           "kernels": "specialised" if spec else "generic"}
    if ctx.dist is not None:  # (a group: world > 1, or the one-rank RCCL rehearsal)
        torch.cuda.synchronize()
        D.barrier(ctx)
        g0 = time.perf_counter()
        allq = D.all_gather_cols(ctx, Q)
        alli = D.all_gather_cols(ctx, it.reshape(1, -1))
        torch.cuda.synchronize()
        out["gather_ms"] = D.max_over_ranks(ctx, [(time.perf_counter() - g0) * 1e3])[0]
        out["gathered_success_rate"] = float((alli <= 64).float().mean())
        assert allq.shape == (8, n * ctx.world)
    return out


def _coll_leg(ctx, stream, n, steps, spec=1, pad=256):
    """Config 5: FK + SDF validity samples of the planner (src/planning.jl collision check):
    Fetch arm (8 joints) with 14 build-defined spheres vs the 7-box fridge scene (door at 2.0 rad,
    base at (1.2, 0, 0)), `n` configurations per GPU, fp32.  Two kernels: min-distance only
    (the RRT validity test) and per-sphere distances + 14x8 gradients (the planner's constraint).
    Multi-GPU: each rank samples its own slice; the validity flags are all-gathered over RCCL
    afterwards (timed separately)."""
    dt = torch.float32
    m, arm, sscc, sdf = fridge_scene()
    plan = sscc.plan(arm, dtype=dt)
    if spec:
        _specialize(plan)
    Q = coll_shard(arm, ctx, n, dt)
    # plain SoA rows padded to ld = n + pad like the FK legs (--row-pad): 2^20-element rows line the
    # 134 row streams of a wave up on the same HBM channels (distances + gradients 104-105 -> 94-96 us,
    # identical results; tools/coll_pad_ab.py, profiles/r03_coll_pad.txt)
    ld = n + pad
    Qb = torch.empty((8, ld), dtype=dt, device=ctx.device)
    Qb[:, :n] = Q
    Qp = Qb[:, :n]
    Dp = torch.zeros((plan.n_sph, ld), dtype=dt, device=ctx.device)[:, :n]
    Gp = torch.zeros((plan.n_sph, 8, ld), dtype=dt, device=ctx.device)[:, :, :n]
    out = {}
    for name, kw in (("min_dist", dict(dists=False, min_dist=True)),
                     ("dists_grads", dict(dists=Dp, grads=Gp))):
        with torch.cuda.stream(stream):
            for _ in range(3):
                r = plan.run(sdf, Qp, stream=stream, **kw)
        torch.cuda.synchronize()
        D.barrier(ctx)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(steps):
            r = plan.run(sdf, Qp, stream=stream, **kw)
        e1.record(stream)
        torch.cuda.synchronize()
        D.barrier(ctx)
        wall, dev_s = D.max_over_ranks(ctx, [time.perf_counter() - t0, e0.elapsed_time(e1) / 1e3])
        ns = plan.n_sph
        nbytes = 8 * 4 + (4 if name == "min_dist" else ns * 4 + ns * 8 * 4)
        out[name] = {"value": n * ctx.world * steps / wall, "unit": "FK+SDF samples/s",
                     "avg_launch_us": dev_s / steps * 1e6, "algorithmic_bytes_per_sample": nbytes,
                     "achieved_GBs": nbytes * n / (dev_s / steps) / 1e9,
                     "layout": f"plain SoA rows, ld = n + {pad}"}
        if name == "min_dist":
            valid = (r[2] > 0).to(torch.uint8).reshape(1, -1)
            out[name]["valid_fraction"] = float(valid.float().mean())
            if ctx.dist is not None:
                torch.cuda.synchronize()
                D.barrier(ctx)
                g0 = time.perf_counter()
                allv = D.all_gather_cols(ctx, valid)
                torch.cuda.synchronize()
                out[name]["gather_ms"] = D.max_over_ranks(ctx, [(time.perf_counter() - g0) * 1e3])[0]
                assert allv.shape[1] == n * ctx.world
    # IneqConst (src/planning.jl:55-68) over n waypoints: margin 0.03, truncation margin + 0.05, one
    # kin_ineq_const_batch launch.  Two inputs: the random samples above, and n / 64 straight-line
    # trajectories of 64 waypoints each (create_straight_trajectory between random start / goal
    # configurations, waypoints of one trajectory side by side) -- the planner's workload, where the
    # broad phase (spheres provably beyond the truncation skip the boxes wave-wide) applies.
    ic = kinhip.IneqConst(sscc, arm, sdf, 1, 0.03, dtype=dt)
    if spec:
        _specialize(ic.plan)
    lo_ = torch.tensor([j.lower_limit for j in arm], dtype=torch.float64)
    hi_ = torch.tensor([j.upper_limit for j in arm], dtype=torch.float64)
    gen = torch.Generator().manual_seed(77 + ctx.rank)
    nt = n // 64
    qs = lo_[:, None] + (hi_ - lo_)[:, None] * torch.rand((8, nt), generator=gen, dtype=torch.float64)
    qg = lo_[:, None] + (hi_ - lo_)[:, None] * torch.rand((8, nt), generator=gen, dtype=torch.float64)
    tt = torch.linspace(0, 1, 64, dtype=torch.float64)
    Qtraj = (qs[:, :, None] + (qg - qs)[:, :, None] * tt).reshape(8, nt * 64).to(dt).to(ctx.device).contiguous()
    ns = plan.n_sph
    nbytes = 8 * 4 + ns * 4 + ns * 8 * 4
    for name, Qx, run in (("ineq_const_random", Q, lambda: ic.eval_batch(Q, stream=stream)),
                          ("ineq_const_trajectories", Qtraj, lambda: ic.eval_batch(Qtraj, stream=stream))):
        with torch.cuda.stream(stream):
            for _ in range(3):
                run()
        torch.cuda.synchronize()
        D.barrier(ctx)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(steps):
            run()
        e1.record(stream)
        torch.cuda.synchronize()
        D.barrier(ctx)
        wall, dev_s = D.max_over_ranks(ctx, [time.perf_counter() - t0, e0.elapsed_time(e1) / 1e3])
        nx = Qx.shape[1]
        out[name] = {"value": nx * ctx.world * steps / wall,
                     "unit": "waypoints/s (values + gradients)" if name.startswith("ineq") else "FK+SDF samples/s",
                     "algorithmic_bytes_per_sample": 36 if name.startswith("min_dist") else nbytes,
                     "avg_launch_us": dev_s / steps * 1e6,
                     "achieved_GBs": (36 if name.startswith("min_dist") else nbytes) * nx / (dev_s / steps) / 1e9}
        if name.startswith("ineq"):
            out[name]["margin"] = 0.03
    # ceiling of the distances + gradients leg (8 rows in, 14 + 112 rows out) from the same run
    pat_c = _pattern_us(8, ns + ns * 8, n, 0, stream, ld=ld)
    out["dists_grads"]["pattern_ceiling_us"] = pat_c
    out["dists_grads"]["frac_of_pattern"] = pat_c / out["dists_grads"]["avg_launch_us"]
    out["dists_grads"]["frac"] = out["dists_grads"]["achieved_GBs"] / HBM_PEAK_GBS
    out["workload"] = (f"fetch arm 8 joints, {plan.n_sph} spheres, fridge scene 7 boxes, {n} configs/GPU, f32, "
                       f"samples sharded across ranks, {'specialised' if spec else 'generic'} kernels")
    return out


def _timed_calls(ctx, stream, fn, reps, warmup=2):
    """(wall s, device s) of `reps` calls of fn on `stream`, bracketed by barrier + synchronize; max over
    ranks.  Device time from HIP events on the launch stream."""
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            out = fn()
    torch.cuda.synchronize()
    D.barrier(ctx)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    with torch.cuda.stream(stream):
        for _ in range(reps):
            out = fn()
    e1.record(stream)
    torch.cuda.synchronize()
    D.barrier(ctx)
    wall, dev_s = D.max_over_ranks(ctx, [time.perf_counter() - t0, e0.elapsed_time(e1) / 1e3])
    return wall, dev_s, out


def _scene_and_coll_ik_legs(ctx, stream, n, steps, spec=1):
    """The two §8 f-rows beside config 5, fp32.
    f2 `UnionSDF(mech)` (src/sdf.jl:14-32, 43-46, 82-97): the fridge's boxes attached to its links
    (kin_sdf_create_attached), one door angle per sample -- fridge_demo.jl's sweep in one launch
    (kin_coll_batch_scene: distances, 14x8 gradients and the minimum; door angle uniform in [0, 2.4],
    fridge at (1.2, 0, 0)).
    f3 bistage collision-aware IK (src/inverse_kinematics.jl:1-21): 4,096 targets per GPU in the open
    fridge's upper compartment (x 0.9..1.05, y +-0.12, z 1.15..1.32, yaw +-0.3), one
    CollisionIKPlan.solve = kin_ik_dls_batch_from + kin_ik_coll_batch (max_iters 128, 3 restarts,
    margin 0.02, the reference's rpy objective)."""
    dt = torch.float32
    m, arm, sscc, sdf = fridge_scene()
    fr = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fridge.urdf"), with_base=True)
    asdf = kinhip.AttachedUnionSDF(fr, [fr.find_joint("door_joint")])
    plan = sscc.plan(arm, dtype=dt)
    scene_const = False
    if spec:
        _specialize(plan)
        try:  # kin_plan_specialize_scene: the fridge's groups, steps and boxes compiled in as well
            plan.specialize_scene(asdf)
            scene_const = True
        except kinhip.KinError as e:
            SPEC_ERRORS.append(str(e)[:300])
    Q = coll_shard(arm, ctx, n, dt, seed=556)
    g = torch.Generator().manual_seed(90 + ctx.rank)
    SQ = torch.zeros((4, n), dtype=torch.float64)
    SQ[0] = torch.rand(n, generator=g, dtype=torch.float64) * 2.4
    SQ[1] = 1.2
    # plain SoA rows padded to ld = n + 256 and preallocated outputs, as config 5's distances + gradients leg
    # (row-aligned 2^20-element streams share HBM channels; a fresh 450 MB output per call starts cold).
    # Back-to-back launches of this kernel slow down in steps under sustained load (a rocprofv3 trace of the
    # bench: 127 us for the first ~1 ms, then 138, 166, 177, settling near 155 us after ~5 ms; the box's power
    # management -- profiles/r05_door_trace.txt); the leg keeps round 4's 3 warm-up launches + 20 timed ones
    pad = 256
    ld = n + pad
    Qb = torch.empty((8, ld), dtype=dt, device=ctx.device)
    Qb[:, :n] = Q
    SQb = torch.empty((4, ld), dtype=dt, device=ctx.device)
    SQb[:, :n] = SQ.to(dt).to(ctx.device)
    Qp, SQp = Qb[:, :n], SQb[:, :n]
    ns = plan.n_sph
    Dp = torch.zeros((ns, ld), dtype=dt, device=ctx.device)[:, :n]
    Gp = torch.zeros((ns, 8, ld), dtype=dt, device=ctx.device)[:, :, :n]
    wall, dev_s, r = _timed_calls(ctx, stream, lambda: plan.run(asdf, Qp, dists=Dp, grads=Gp, min_dist=True,
                                                                scene_q=SQp, stream=stream), steps, warmup=3)
    nbytes = (8 + 4) * 4 + ns * 4 + ns * 8 * 4 + 4  # q + scene columns in; distances, gradients, minimum out
    out = {"f2_scene_door_sweep": {"value": n * ctx.world * steps / wall, "unit": "FK+SDF samples/s",
                                   "avg_launch_us": dev_s / steps * 1e6, "algorithmic_bytes_per_sample": nbytes,
                                   "achieved_GBs": nbytes * n / (dev_s / steps) / 1e9,
                                   "valid_fraction": float((r[2] > 0).float().mean()),
                                   "kernel": ("kinhip_jit_collc_1 (specialised, the fridge's tables compiled in)"
                                              if scene_const else
                                              "kinhip_jit_colls_1_2 (specialised, 2 scene groups)" if spec else "k_coll_scene"),
                                   "layout": f"plain SoA rows, ld = n + {pad}, preallocated outputs"}}
    # the access pattern's ceiling (12 rows in, 14 + 112 rows out; the minimum's row aside)
    pat = _pattern_us(12, ns + ns * 8, n, 0, stream, ld=ld)
    out["f2_scene_door_sweep"]["pattern_ceiling_us"] = pat
    out["f2_scene_door_sweep"]["frac_of_pattern"] = pat / out["f2_scene_door_sweep"]["avg_launch_us"]
    gl = m.find_link("gripper_link")
    nt = 4096
    rng = np.random.default_rng(17 + ctx.rank)
    tg = np.zeros((12, nt))
    for k in range(nt):
        x, y, z, yaw = rng.uniform(0.9, 1.05), rng.uniform(-0.12, 0.12), rng.uniform(1.15, 1.32), rng.uniform(-0.3, 0.3)
        c, s_ = np.cos(yaw), np.sin(yaw)
        R = np.array([[c, -s_, 0.0], [s_, c, 0.0], [0.0, 0.0, 1.0]])
        tg[:, k] = np.concatenate([R.T.reshape(-1), [x, y, z]])
    tg = torch.tensor(tg, dtype=dt, device=ctx.device).contiguous()
    cplan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=dt)
    if spec:
        _specialize(cplan)
    Q0 = torch.zeros((8, nt), dtype=dt, device=ctx.device)
    reps = 5
    wall, dev_s, (Qs, it, err) = _timed_calls(
        ctx, stream, lambda: cplan.solve(sdf, tg, Q0, max_iters=128, restarts=3, seed=1, index_base=ctx.rank * nt,
                                         stream=stream), reps, warmup=1)
    conv = it <= 128
    out["f3_collision_ik"] = {"value": nt * ctx.world * reps / wall, "unit": "bistage IK solves/s",
                              "targets_per_gpu": nt, "ms_per_batch": dev_s / reps * 1e3,
                              "stage2_attempt1": "from the stage-1 start pose (kin_ik_coll_batch_alt)",
                              "converged": float(conv.float().mean()),
                              "min_sphere_distance_converged": float(err[2][conv].min()) if bool(conv.any()) else None,
                              "kernels": "specialised" if spec else "generic"}
    # the two stages apart: stage 2 alone from stage 1's answers (kin_ik_coll_batch)
    kw = dict(max_iters=128, restarts=3, seed=1, with_rot=2, index_base=ctx.rank * nt)
    Q1 = torch.empty_like(Q0)
    cplan.ik_dls(tg, Q1, Q0=Q0, **kw)
    Q2 = torch.empty_like(Q0)
    _, dev2, _ = _timed_calls(ctx, stream, lambda: cplan.ik_coll(sdf, tg, Q2, Q0=Q1, margin=0.02, stream=stream,
                                                                 Q_alt=Q0, **kw), reps, warmup=1)
    out["f3_collision_ik"]["ms_stage2"] = dev2 / reps * 1e3
    out["f3_collision_ik"]["ms_stage1"] = out["f3_collision_ik"]["ms_per_batch"] - dev2 / reps * 1e3
    # the same bistage solve against UnionSDF(fridge) attached to its mechanism, the door angle per target
    # (kin_ik_coll_batch_scene; test/test_inverse_kinematics.jl:52-86, fridge_demo.jl's door)
    SQ2 = torch.zeros((4, nt), dtype=torch.float64)
    SQ2[0] = torch.rand(nt, generator=g, dtype=torch.float64) * 0.9 + 1.5
    SQ2[1] = 1.2
    SQ2 = SQ2.to(dt).to(ctx.device).contiguous()
    out["f3_collision_ik_scene_door"] = _bistage_leg(ctx, stream, cplan, asdf, tg, Q0, nt, reps, scene_q=SQ2,
                                                     spec=spec)
    out["f3_pr2_collision_ik"] = _pr2_leg(ctx, stream, asdf, nt, reps, spec)
    for n_p in (4096, 65536):
        out[f"f3_collision_ik_pillar_{n_p}"] = _pillar_leg(ctx, stream, m, arm, sscc, sdf, n_p, spec)
    return out


def _bistage_leg(ctx, stream, cplan, sdf, tg, Q0, nt, reps, scene_q=None, spec=1):
    """One CollisionIKPlan.solve per batch (stage 1 kin_ik_dls_batch_from + stage 2, its restart attempt 1 from
    Q0: kin_ik_coll_batch_alt), timed, and stage 2 alone from stage 1's answers."""
    kw = dict(max_iters=128, restarts=3, seed=1, with_rot=2, index_base=ctx.rank * nt)
    wall, dev_s, (Qs, it, err) = _timed_calls(
        ctx, stream, lambda: cplan.solve(sdf, tg, Q0, stream=stream, scene_q=scene_q, **kw), reps, warmup=1)
    conv = it <= 128
    Q1 = Q0.clone()
    cplan.ik_dls(tg, Q1, Q0=Q0, **kw)
    Q2 = torch.empty_like(Q0)
    _, dev2, _ = _timed_calls(ctx, stream, lambda: cplan.ik_coll(sdf, tg, Q2, Q0=Q1, margin=0.02, stream=stream,
                                                                 scene_q=scene_q, Q_alt=Q0, **kw), reps, warmup=1)
    return {"value": nt * ctx.world * reps / wall, "unit": "bistage IK solves/s", "targets_per_gpu": nt,
            "ms_per_batch": dev_s / reps * 1e3, "ms_stage2": dev2 / reps * 1e3,
            "converged": float(conv.float().mean()),
            "min_sphere_distance_converged": float(err[2][conv].min()) if bool(conv.any()) else None,
            "kernels": "specialised" if spec else "generic"}


def _pr2_leg(ctx, stream, asdf, nt, reps, spec):
    """The reference's own collision-aware IK shape (test/test_inverse_kinematics.jl:52-86, fridge_demo.jl):
    PR2 (tests/golden/pr2_two_arms.urdf) with its planar base, joints = vcat(rarm, larm) -- 14 joints + base =
    17 variables -- spheres on both arms' collision links, the l_gripper_tool_frame target inside the fridge
    (Transform((0, 0, 1.2)) * pose_fridge, jittered), the door angle per target, from reset_manip_pose.  fp32."""
    dt = torch.float32
    m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "pr2_two_arms.urdf"), with_base=True)
    joints = [m.find_joint(n) for n in kinhip.PR2_RARM_JOINTS + kinhip.PR2_LARM_JOINTS]
    m.set_joint_angles([m.find_joint("torso_lift_joint")], [0.3, 0.0, 0.0, 0.0])
    sscc = kinhip.SweptSphereCollisionChecker(m)
    for name, c, r in kinhip.PR2_ARM_SPHERES:
        sscc.add_coll_sphere(m.find_link(name), c, r)
    cplan = kinhip.CollisionIKPlan(sscc, m.find_link("l_gripper_tool_frame"), joints, dtype=dt)
    if spec:
        _specialize(cplan)
    r, l, _ = kinhip.PR2_MANIP_POSE
    q0 = np.concatenate([np.deg2rad(np.array(r + l)), np.zeros(3)])
    Q0 = torch.tensor(np.repeat(q0[:, None], nt, 1), dtype=dt, device=ctx.device).contiguous()
    rng = np.random.default_rng(29 + ctx.rank)
    tg = np.zeros((12, nt))
    for k in range(nt):
        yaw = rng.uniform(-0.2, 0.2)
        c, s_ = np.cos(yaw), np.sin(yaw)
        R = np.array([[c, -s_, 0.0], [s_, c, 0.0], [0.0, 0.0, 1.0]])
        tg[:, k] = np.concatenate([R.T.reshape(-1), [1.2 + rng.uniform(-0.06, 0.0), rng.uniform(-0.06, 0.06),
                                                     1.2 + rng.uniform(-0.05, 0.05)]])
    tg = torch.tensor(tg, dtype=dt, device=ctx.device).contiguous()
    SQ = torch.zeros((4, nt), dtype=torch.float64)
    SQ[0] = torch.tensor(rng.uniform(1.6, 2.4, nt))
    SQ[1] = 1.2
    SQ = SQ.to(dt).to(ctx.device).contiguous()
    out = _bistage_leg(ctx, stream, cplan, asdf, tg, Q0, nt, reps, scene_q=SQ, spec=spec)
    out["variables"] = cplan.n_qcols
    return out


def _pillar_leg(ctx, stream, m, arm, sscc, sdf0, nt, spec, reps=5):
    """Stage 2 where it works: tests/test_gpu_collision_ik.py's pillar scene -- a box
    (8 cm) on elbow_flex_link of the collision-free solution for the target (0.75, 0.15, 1.0), targets
    jittered by +-5 mm, so stage 1's answers collide for most of them -- `nt` targets per GPU, fp32;
    stage 1 once (kin_ik_dls_batch_from), then stage 2 (kin_ik_coll_batch) timed: stage-2 solves/s."""
    dt = torch.float32
    gl = m.find_link("gripper_link")
    T0 = np.eye(4)
    T0[:3, 3] = (0.75, 0.15, 1.0)
    m.set_joint_angles(arm, np.zeros(8))
    kinhip.inverse_kinematics_(m, gl, arm, T0)
    P = np.eye(4)
    P[:3, 3] = kinhip.get_transform(m, m.find_link("elbow_flex_link"))[:3, 3]
    m.set_joint_angles(arm, np.zeros(8))
    sdf = kinhip.UnionSDF(sdf0.sdfs + [kinhip.BoxSDF(P, (0.08, 0.08, 0.08))])
    rng = np.random.default_rng(5 + ctx.rank)
    tg = np.zeros((12, nt))
    for k in range(nt):
        t = np.asarray(T0[:3, 3]) + rng.uniform(-0.005, 0.005, 3)
        tg[:, k] = np.concatenate([np.eye(3).reshape(-1), t])
    tg = torch.tensor(tg, dtype=dt, device=ctx.device).contiguous()
    cplan = kinhip.CollisionIKPlan(sscc, gl, arm, dtype=dt)
    if spec:
        _specialize(cplan)
    kw = dict(max_iters=128, restarts=3, seed=1, with_rot=2, index_base=ctx.rank * nt)
    Q0 = torch.zeros((8, nt), dtype=dt, device=ctx.device)
    Q1 = torch.empty_like(Q0)
    cplan.ik_dls(tg, Q1, Q0=Q0, **kw)
    _, _, D1 = sscc.plan(arm, dtype=dt).run(sdf, Q1, dists=False, min_dist=True)
    Q2 = torch.empty_like(Q0)
    wall, dev_s, (Q2, it, err) = _timed_calls(
        ctx, stream, lambda: cplan.ik_coll(sdf, tg, Q2, Q0=Q1, margin=0.02, stream=stream, **kw), reps, warmup=1)
    conv = it <= 128
    return {"value": nt * ctx.world * reps / wall, "unit": "stage-2 solves/s (kin_ik_coll_batch)",
            "targets_per_gpu": nt, "ms_per_batch": dev_s / reps * 1e3,
            "stage1_answers_under_margin": float((D1 < 0.02).float().mean()),
            "converged": float(conv.float().mean()),
            "min_sphere_distance_converged": float(err[2][conv].min()) if bool(conv.any()) else None,
            "kernels": "specialised" if spec else "generic"}


def _nakamura_leg(m, arm, gl, ctx, stream, n=1 << 18, reps=5, spec=1):
    """point_inverse_kinematics_nakamura (50 SR-inverse iterations, the reference's
    `.+ 1.0` quirk), fp64 as the reference, `n` reachable points per GPU from q0 = 0."""
    dt = torch.float64
    plan = m.plan(arm, out_links=[gl], jac_link=gl, jac_joints=arm, with_rot=False, dtype=dt)
    if spec:
        _specialize(plan)
    start, cnt = D.shard_range(n, ctx.rank)
    Qt = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], cnt, start=start,
                                seed=99, dtype=dt, device=ctx.device)
    fk = m.plan(arm, out_links=[gl], dtype=dt)  # generic FK-only plan for targets / residuals
    pts = fk.run(Qt)[0][0][9:12].contiguous()
    Qs = [torch.zeros((8, cnt), dtype=dt, device=ctx.device) for _ in range(reps + 1)]
    with torch.cuda.stream(stream):
        plan.point_ik_nakamura(pts, Qs[0], stream=stream)
    torch.cuda.synchronize()
    D.barrier(ctx)
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for k in range(1, reps + 1):
            plan.point_ik_nakamura(pts, Qs[k], stream=stream)
    torch.cuda.synchronize()
    D.barrier(ctx)
    wall = D.max_over_ranks(ctx, [time.perf_counter() - t0])[0]
    got = fk.run(Qs[-1])[0][0][9:12]
    err = (got - pts).norm(dim=0)
    return {"value": n * ctx.world * reps / wall, "unit": "point-IK solves/s (50 iterations each)",
            "points_per_gpu": n, "ms_per_batch": wall / reps * 1e3, "dtype": "f64",
            "median_residual_m": float(err.median()), "kernels": "specialised" if spec else "generic"}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_baseline(m, N_budget_s=12.0, single_s=4.0):
    """Reference-faithful C restatement (oracle/kin_oracle.c) on the host cores, bounded sample:
    all-threads run (the reported value) and a 1-thread run (1 core and all cores)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    tree = O.parse_urdf_tree(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
    om = O.OracleMech(tree)
    ids = [tree.joint_id(n) for n in ARM]
    gl = tree.link_id("gripper_link")
    # every host core this process can use (SURVEY.md 8d "all host cores"): the affinity set, capped by
    # the container's CPU quota (cgroup cpu.max) -- on the GPU box the affinity set is the whole machine
    # (256) but the quota is 16 CPUs, and 256 threads throttled onto 16 CPUs run 40x slower than 16
    # (measured: 3.3e5 vs 1.3e7 evals/s).  KIN_CPU_THREADS overrides.
    quota = _cgroup_cpu_max()
    usable = len(os.sched_getaffinity(0))
    if isinstance(quota, float):
        usable = max(1, min(usable, int(quota + 0.5)))
    threads = int(os.environ.get("KIN_CPU_THREADS", usable))
    arm = [m.find_joint(n) for n in ARM]
    chunk = 1 << 16
    q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], chunk,
                               dtype=torch.float64).numpy()

    def run(nthr, budget, n):
        om.fk_jac_batch(q[:, :1024], ids, gl, ids, True, False, n_threads=nthr)  # warm
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget:
            om.fk_jac_batch(q[:, :n], ids, gl, ids, True, False, n_threads=nthr)
            done += n
        return done, time.perf_counter() - t0

    done, dt = run(threads, N_budget_s, chunk)
    d1, t1 = run(1, single_s, 4096)
    return {"value": done / dt, "unit": "evals/s", "cores": threads, "kind": "port",
            "single_core_value": d1 / t1, "cpu_model": _cpu_model(), "host_cpus_visible": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_max": _cgroup_cpu_max(),
            "sample": f"{done} Fetch configs (chunks of {chunk}) through or_fk_jac_batch: per-config "
                      f"Mechanism state, cache invalidate, quaternion joint transforms, dense 4x4 fp64 "
                      f"(src/algorithm.jl restated), {threads} OpenMP threads, {dt:.1f} s; plus {d1} configs "
                      f"on 1 thread in {t1:.1f} s"}


def _cgroup_cpu_max():
    """The container's CPU quota (cgroup v2 cpu.max: "quota period" or "max period"), if readable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
        return "unlimited" if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        return None


def _copy_bw(dev, nbytes=1 << 31):
    """Device-to-device copy rate (read + write bytes / s) as the practical HBM ceiling."""
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2 * nbytes * 10 / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    return gbs


def _pmc_valu(fname):
    """Issue-based VALU busy of a committed PMC summary (tools/summarize_prof.py), for the legs whose
    bound is VALU / latency rather than HBM (configs 4 and 5)."""
    for rnd in ("r05_", "r04_", "r03_", "r02_"):  # the newest committed round's summary
        p = os.path.join(ROOT, "profiles", rnd + fname)
        if os.path.exists(p):
            fname = rnd + fname
            break
    else:
        return None
    with open(p) as f:
        d = json.load(f)
    v = d.get("valu", {})
    return {"valu_busy": v.get("valu_busy"), "valu_insts_per_wave": v.get("valu_insts_per_wave"),
            "traffic_over_algorithmic": d.get("traffic_over_algorithmic"), "source": "profiles/" + fname}


def _pmc_traffic(workload, fname="pmc_fk_jac_f32.json"):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/), if present."""
    p = os.path.join(ROOT, "profiles", fname)
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_launch")
    return None


_PROBE = None


# the probe's occupancy sweep: (dynamic LDS bytes, lanes) per workgroup -- as many waves as registers allow,
# then 20, 16, 12, 8, 6 and 4 waves per CU (160 KB of LDS per CU)
PROBE_OCC = ((0, 256), (32768, 256), (40960, 256), (53248, 256), (65536, 256), (53248, 128), (65536, 128))


def _pattern_us(rows_in, rows_out, n, tile, stream, reps=20, warmup=3, ld=0, per_lane=1):
    """The fastest of the access pattern's runs over the PROBE_OCC occupancies (_pattern_at)."""
    return min(_pattern_at(rows_in, rows_out, n, tile, stream, reps, warmup, ld, per_lane, lds, blk)
               for lds, blk in PROBE_OCC)


def _pattern_at(rows_in, rows_out, n, tile, stream, reps=20, warmup=3, ld=0, per_lane=1, lds=0, blk=256):
    """The access pattern of a leg with no arithmetic (kinematics.jl_amd/lib/libkinprobe.so, a measurement
    probe built beside the engine): rows_in rows of q read and rows_out rows written per configuration,
    fp32, tiled SoA (tile > 0) or plain rows (tile = 0) `ld` >= n elements apart (0: ld = n), addressed as
    the kernels address them (per-row buffer descriptors, 32-bit lane offsets, uniform tile divide,
    non-temporal stores; per_lane > 1: launch_fk's grid-strided form), `lds` bytes of unused LDS per
    workgroup of `blk` lanes capping its occupancy.  Average launch time (µs) from HIP events on `stream`: the leg's
    ceiling measured in the same run."""
    global _PROBE
    import ctypes as C
    if _PROBE is None:
        _PROBE = C.CDLL(os.path.join(ROOT, "kinematics.jl_amd", "lib", "libkinprobe.so"))
        _PROBE.kinprobe_pattern4.argtypes = [C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int,
                                             C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        _PROBE.kinprobe_pattern4.restype = C.c_int
    ld = tile if tile else (ld or n)
    ntot = -(-n // tile) * tile if tile else ld
    q = torch.zeros(rows_in * ntot, dtype=torch.float32, device=stream.device)
    out = torch.zeros(rows_out * ntot, dtype=torch.float32, device=stream.device)
    st = stream.cuda_stream

    def launch():
        rc = _PROBE.kinprobe_pattern4(rows_in, rows_out, n, tile, ld, per_lane, lds, blk, q.data_ptr(), out.data_ptr(),
                                      st)
        assert rc == 0, rc
    for _ in range(warmup):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    del q, out
    return us


def _cold_leg(leg, n, stream, bytes_per_eval, reps=10, tiled=True):
    """One launch at a time after a 1 GiB read (torch sum) has evicted the Infinity Cache: the
    launch's own HIP events bracket it alone (the read is outside them).  `leg`: (plan, q, poses, jac)
    in the tiled layout (kin_plan_run_tiled) or, with tiled=False, plain SoA rows (kin_plan_run)."""
    plan, Qt, P, J = leg

    def run():
        if tiled:
            plan.run_tiled(Qt, n, P, J, stream=stream)
        else:
            plan.run(Qt, P, J, stream=stream)
    scrub = torch.ones(1 << 28, dtype=torch.float32, device=Qt.device)
    e = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    with torch.cuda.stream(stream):
        run()
        for e0, e1 in e:
            scrub.sum()
            e0.record(stream)
            run()
            e1.record(stream)
    torch.cuda.synchronize()
    t = sum(a.elapsed_time(b) for a, b in e) / reps / 1e3
    ach = bytes_per_eval * n / t / 1e9
    del scrub, plan, Qt, P, J
    return {"avg_launch_us": t * 1e6, "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS,
            "method": "each launch after a 1 GiB read of another buffer (Infinity Cache evicted), 10 launches"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--n", type=int, default=1 << 20, help="configurations per GPU")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--extras", type=int, default=1, help="also time fp64 FK+J, config 2, IK and collision legs")
    ap.add_argument("--row-pad", type=int, default=256, help="elements of padding per SoA row (ld = n + pad)")
    ap.add_argument("--layout", choices=["tiled", "soa"], default="tiled",
                    help="headline layout: tiled SoA (kin_plan_run_tiled) or plain SoA rows (kin_plan_run)")
    ap.add_argument("--tile", type=int, default=8192, help="configurations per tile of the tiled layout")
    ap.add_argument("--layout64", choices=["tiled", "soa"], default="tiled", help="layout of the fp64 legs")
    ap.add_argument("--spec", type=int, default=1,
                    help="1: plan-specialised kernels (kin_plan_specialize), 0: the generic kernels")
    ap.add_argument("--sweep", action="store_true", help="batch-size sweep, unpadded rows, strong scaling")
    args = ap.parse_args()

    # stdout carries the one JSON line only: RCCL prints its version banner to the process's stdout when the
    # group initialises (a round-6 one-rank RCCL run had four such lines before the JSON), so until the line is
    # printed file descriptor 1 points at stderr
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    # KINHIP_DIST_ALWAYS_GROUP=1 (torchrun --nproc-per-node 1): a one-rank RCCL group runs every
    # collective of the sharded path -- barriers, max over ranks, the result gathers, the strong-scaling
    # leg -- on the single-GPU box, exactly as each rank of an N-GPU run does
    ctx = D.init_from_env(always_group=os.environ.get("KINHIP_DIST_ALWAYS_GROUP") == "1")
    rank, ws, dev = ctx.rank, ctx.world, ctx.device
    m = kinhip.parse_urdf(os.path.join(ROOT, "tests", "golden", "fetch.urdf"))
    arm = [m.find_joint(n) for n in ARM]
    gl = m.find_link("gripper_link")
    N = args.n
    lo, hi = [j.lower_limit for j in arm], [j.upper_limit for j in arm]
    stream = torch.cuda.Stream(dev)

    def mkplan(dtype, jac, links, spec):
        plan = m.plan(arm, out_links=links, jac_link=gl if jac else None, jac_joints=arm if jac else None,
                      with_rot=True, dtype=dtype)
        return _specialize(plan) if spec else plan

    def leg(dtype, jac, links, n=N, pad=args.row_pad, start=None, spec=args.spec):
        """Device-resident SoA buffers; every row padded to ld = n + pad elements (the C-ABI's
        ldq / ldp / ldj): rows exactly 2^k elements apart line all 68 streams of a wave up on the
        same HBM channels (tools/ld_probe.py, profiles/r01_row_pad_probe.txt)."""
        plan = mkplan(dtype, jac, links, spec)
        ld = n + pad
        Qb = torch.empty((8, ld), dtype=dtype, device=dev)
        Qb[:, :n] = kinhip.uniform_configs(lo, hi, n, start=rank * n if start is None else start, dtype=dtype,
                                           device=dev)
        poses = torch.zeros((len(links), 12, ld), dtype=dtype, device=dev)[:, :, :n]
        J = torch.zeros((8, 6, ld), dtype=dtype, device=dev)[:, :, :n] if jac else None
        return plan, Qb[:, :n], poses, J

    def leg_tiled(dtype, jac, links, tile, n=N, start=None, spec=args.spec):
        """Tiled SoA (kin_plan_run_tiled): (ntiles, rows, tile) arrays, one contiguous run per
        output row and tile."""
        plan = mkplan(dtype, jac, links, spec)
        Q = kinhip.uniform_configs(lo, hi, n, start=rank * n if start is None else start, dtype=dtype, device=dev)
        Qt = kinhip.tiled(Q, tile)
        nt = Qt.shape[0]
        # zero-filled: the output pages are touched (mapped) before the first timed launch
        poses = torch.zeros((nt, len(links), 12, tile), dtype=dtype, device=dev)
        J = torch.zeros((nt, 8, 6, tile), dtype=dtype, device=dev) if jac else None
        return plan, Qt, poses, J

    def timed_leg(dtype, jac, links, layout, n=N, start=None, steps=args.steps, warmup=args.warmup):
        """(wall s, device s) of `steps` launches of one FK(+J) workload in `layout`:
        "tiled" / "tileT" (kin_plan_run_tiled) or "soa" / "soa_padP" (kin_plan_run); a "generic_"
        prefix runs the generic (not plan-specialised) kernel."""
        spec = args.spec
        if layout.startswith("generic_"):
            spec, layout = 0, layout[8:]
        if layout.startswith("tile"):
            tile = args.tile if layout == "tiled" else int(layout[4:])
            plan, Qx, Px, Jx = leg_tiled(dtype, jac, links, tile, n=n, start=start, spec=spec)
            r = _time_tiled(plan, Qx, n, Px, Jx, steps, warmup, ctx, stream)
        else:
            pad = args.row_pad if layout == "soa" else int(layout[7:])
            plan, Qx, Px, Jx = leg(dtype, jac, links, n=n, pad=pad, start=start, spec=spec)
            r = _time_plan(plan, Qx, Px, Jx, steps, warmup, ctx, stream)
        del plan, Qx, Px, Jx
        return r

    # ---- headline: FK + J, fp32 -------------------------------------------------
    wall, dev_s = timed_leg(torch.float32, True, [gl], args.layout)
    headline_spec = bool(args.spec) and not SPEC_ERRORS
    evals = N * ws * args.steps
    value = evals / wall
    bytes_per_eval = (8 + 12 + 48) * 4  # q in + pose + J out (algorithmic)
    t_launch = dev_s / args.steps
    achieved = bytes_per_eval * N / t_launch / 1e9
    traffic = _pmc_traffic(("fkjac32t" if args.layout == "tiled" else "fkjac32") + ("s" if headline_spec else ""))
    out = {
        "metric": "FK+Jacobian evals/sec, Fetch URDF, batch=1M, at 1/2/4/8 MI355X",
        "value": value, "unit": "evals/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (counter-hashed uniform joint angles within "
                                                       "fetch.urdf limits, seed 20261015)",
        "config": {"workload": "fetch_fk_jac_gripper_link (BASELINE configs[2])", "urdf": "fetch",
                   "batch_per_gpu": N, "global_batch": N * ws, "q_joints": 8, "jacobian": "6x8 geometric",
                   "parallelism": f"dp{ws} (independent shards)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "kinhip_jit_fk_f32_<program hash> (k_fk body specialised to the plan)" if headline_spec else
                     "k_fk<float, 8>", "algorithmic_bytes_per_eval": bytes_per_eval,
                     "avg_launch_us": t_launch * 1e6},
    }
    out["config"]["dist_backend"] = ctx.backend  # "nccl" = RCCL on ROCm; "none": one process, no group
    out["config"]["kernels"] = ("plan-specialised (kin_plan_specialize: program constants folded by hiprtc)"
                                if headline_spec else "generic (program read from device memory)")
    if args.layout == "tiled":
        out["config"]["layout"] = (f"tiled SoA, tile {args.tile} (kin_plan_run_tiled: Julia Array{{Float32,3}}"
                                   f"({args.tile}, rows, N/{args.tile}))")
    else:
        out["config"]["layout"] = f"plain SoA (kin_plan_run), rows padded to ld = N + {args.row_pad}"
    out["roofline"]["traffic_source"] = ("profiles/pmc_fk_jac_f32.json: rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this "
                                         "workload (2*FETCH_SIZE + WRITE_SIZE, gfx950), committed with the round's "
                                         "profiles" if traffic else None)
    if args.extras:
        out["roofline"]["torch_copy_GBs"] = _copy_bw(dev)  # context: torch device-to-device copy rate
        # the same bytes in the same layout with no kinematics (8 rows read, 60 written): this leg's ceiling
        pat = _pattern_us(8, 60, N, args.tile if args.layout == "tiled" else 0, stream, ld=N + args.row_pad)
        out["roofline"]["pattern_ceiling"] = {"avg_launch_us": pat, "frac_of_pattern": pat / (t_launch * 1e6),
                                              "achieved_GBs": bytes_per_eval * N / pat / 1e3,
                                              "probe": "kinprobe_pattern4(8 in, 60 out, same layout and addressing), fastest over occupancies, same run"}
        # The 2^20 working set (q + outputs, 285 MB) is about the 256 MiB Infinity Cache, so back-to-back
        # launches find part of the previous launch's lines on die.  Two checks beside the headline:
        # the same launch after a 1 GiB read has evicted the cache (cold), and batches 4x and 16x the
        # Infinity Cache, where nothing survives between launches.
        if args.layout == "tiled":
            out["roofline"]["cold_cache"] = _cold_leg(leg_tiled(torch.float32, True, [gl], args.tile), N, stream,
                                                      bytes_per_eval)
            big = {}
            for lg, k_s in ((22, 10), (24, 5)):
                w_b, d_b = timed_leg(torch.float32, True, [gl], args.layout, n=1 << lg, steps=k_s, warmup=2)
                ach = bytes_per_eval * (1 << lg) / (d_b / k_s) / 1e9
                pat_b = _pattern_us(8, 60, 1 << lg, args.tile, stream, reps=k_s, warmup=1, per_lane=1)
                big[f"2^{lg}"] = {"evals_per_s": (1 << lg) * ws * k_s / w_b, "avg_launch_us": d_b / k_s * 1e6,
                                  "achieved_GBs": ach, "frac": ach / HBM_PEAK_GBS,
                                  "pattern_ceiling_us": pat_b, "frac_of_pattern": pat_b / (d_b / k_s * 1e6),
                                  "working_set_MB": bytes_per_eval * (1 << lg) / 1e6,
                                  "kernel": "as the headline (fp32 runs the one-per-lane grid at every size)"}
            out["roofline"]["large_batches"] = big
            out["roofline"]["rocprof_note"] = ("the cold-cache and 2^22 legs launch the headline kernel too (same name); "
                                               "tools/trace_headline.py splits a rocprofv3 kernel trace of this bench "
                                               "per leg (profiles/r02_bench_trace_legs.json: the 50 timed launches)")
    if args.extras and headline_spec:
        # the same workload through the most literal form of the API: generic kernel (no run-time
        # compilation), plain column-major rows (padded ld) -- kin_plan_run as a Julia caller would
        # use it first; its kernel (k_fk<float, 8>) is profiled apart from the headline's
        wg, dg = timed_leg(torch.float32, True, [gl], "generic_soa")
        out["fk_jac_f32_generic_plain_soa"] = {"value": N * ws * args.steps / wg, "unit": "evals/s",
                                               "avg_launch_us": dg / args.steps * 1e6,
                                               "achieved_GBs": bytes_per_eval * N / (dg / args.steps) / 1e9}
    if args.extras:
        # the layout the Julia shim's get_jacobian! hands over (KinematicsHIP.jl: ROCMatrix(N, 8) /
        # ROCArray(N, 6, 8) -> plain SoA rows with ld = N, unpadded), warm like the headline and cold
        wj, dj = timed_leg(torch.float32, True, [gl], "soa_pad0")
        aj = bytes_per_eval * N / (dj / args.steps) / 1e9
        out["fk_jac_f32_julia_layout"] = {
            "value": N * ws * args.steps / wj, "unit": "evals/s", "avg_launch_us": dj / args.steps * 1e6,
            "achieved_GBs": aj, "frac": aj / HBM_PEAK_GBS, "vs_headline": (N * ws * args.steps / wj) / value,
            "layout": "plain SoA, ld = N (unpadded)",
            "kernels": "specialised" if headline_spec else "generic",
            "cold_cache": _cold_leg(leg(torch.float32, True, [gl], pad=0), N, stream, bytes_per_eval, tiled=False)}
    if args.sweep:
        # the same workload in the other layouts: plain SoA (padded and unpadded rows), other tiles
        lay = {}
        for name in ("soa_pad%d" % args.row_pad, "soa_pad0", "tile2048", "tile4096", "tile8192",
                     "generic_soa_pad%d" % args.row_pad, "generic_tile4096", "generic_tile8192"):
            wt, dt_ = timed_leg(torch.float32, True, [gl], name)
            lay[name] = {"value": N * ws * args.steps / wt, "unit": "evals/s", "avg_launch_us": dt_ / args.steps * 1e6,
                         "achieved_GBs": bytes_per_eval * N / (dt_ / args.steps) / 1e9}
        out["fk_jac_f32_layouts"] = lay
        for name in ("generic_soa", "generic_tile4096", "soa", "tile8192"):  # fp64: the layout matters more
            w_, d_ = timed_leg(torch.float64, True, [gl], name, steps=max(5, args.steps // 2), warmup=3)
            lay[name + "_f64"] = {"value": N * ws * max(5, args.steps // 2) / w_, "unit": "evals/s",
                                  "avg_launch_us": d_ / max(5, args.steps // 2) * 1e6,
                                  "achieved_GBs": 544 * N / (d_ / max(5, args.steps // 2)) / 1e9}
    if args.sweep:
        # batch sweep: launch-overhead vs bandwidth regime, fp32 FK + J
        sweep = {}
        for lg in range(16, 27, 2):
            for name in ("soa_pad0", "soa_pad%d" % args.row_pad, "tile%d" % args.tile):
                n_s = 1 << lg
                k_s = max(5, min(50, (1 << 26) // n_s))
                ws_, ds_ = timed_leg(torch.float32, True, [gl], name, n=n_s, steps=k_s, warmup=3)
                sweep[f"2^{lg} {name}"] = {"evals_per_s": n_s * ws * k_s / ws_, "avg_launch_us": ds_ / k_s * 1e6,
                                           "achieved_GBs": bytes_per_eval * n_s / (ds_ / k_s) / 1e9}
        out["batch_sweep_fk_jac_f32"] = sweep
    if ctx.dist is not None:  # strong scaling: one global 2^20 batch split across the ranks
        st0, cnt = D.split_range(N, rank, ws)
        w_s, d_s = timed_leg(torch.float32, True, [gl], args.layout, n=cnt, start=st0)
        out["strong_scaling_fk_jac_f32"] = {"global_batch": N, "value": N * args.steps / w_s, "unit": "evals/s",
                                            "ms_per_step": w_s / args.steps * 1e3}
    if args.extras:
        # fp64 FK+J (reference precision) and config 2 (FK of 6 links, fp64)
        k2 = max(5, args.steps // 2)
        # (fp64 rows are 8 B per lane: the tiled layout keeps each output row of a workgroup in one
        # run and is 10-13% faster here than plain rows, fk_jac_f32_layouts *_f64)
        lay64 = "tile%d" % (args.tile // 2) if args.layout64 == "tiled" else "soa"  # same bytes per tile row
        w64, d64 = timed_leg(torch.float64, True, [gl], lay64, steps=k2, warmup=3)
        a64 = 544 * N / (d64 / k2) / 1e9
        out["fp64_fk_jac"] = {"value": N * ws * k2 / w64, "unit": "evals/s", "avg_launch_us": d64 / k2 * 1e6,
                              "achieved_GBs": a64, "layout": lay64,
                              "roofline": {"bound": "hbm", "achieved": a64, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                           "frac": a64 / HBM_PEAK_GBS,
                                           "traffic": _pmc_traffic("fkjac64ts", "pmc_fk_jac_f64.json"),
                                           "kernel": "kinhip_jit_fk_f64_<program hash>" if args.spec else
                                           "k_fk<double, 8>", "algorithmic_bytes_per_eval": 544,
                                           "working_set_MB": 544 * N / 1e6}}
        links = [m.find_link(n) for n in EXAMPLE_LINKS]
        w2, d2 = timed_leg(torch.float64, False, links, lay64, steps=k2, warmup=3)
        out["config2_fk6_f64"] = {"value": N * ws * k2 / w2, "unit": "evals/s", "avg_launch_us": d2 / k2 * 1e6,
                                  "achieved_GBs": (8 + 72) * 8 * N / (d2 / k2) / 1e9, "layout": lay64}
        out["config4_ik_dls"] = _ik_leg(m, arm, gl, ctx, stream, spec=args.spec)
        out["config4_ik_dls"]["pmc"] = _pmc_valu("pmc_ik32s.json")
        # the reference's own objective (src/inverse_kinematics.jl:38-50: [p* - p; rpy* - rpy], rpy_jac)
        # (with the error-scaled damping: the rpy residual converges worse on a fixed lambda -- 0.992 success
        # at max_step 0.5, 0.997 damped, profiles/r04_bench_k.json)
        out["config4_ik_dls_rpy"] = _ik_leg(m, arm, gl, ctx, stream, spec=args.spec,
                                            over=dict(IK_KW_DAMPED, with_rot=2))
        # the error-scaled damping (kin_ik_params.damp_err) for comparison
        out["config4_ik_dls_damped"] = _ik_leg(m, arm, gl, ctx, stream, spec=args.spec,
                                               over=dict(max_step=1.0, damp_err=0.01))
        out["ik_dls_1M_targets"] = _ik_leg(m, arm, gl, ctx, stream, n=1 << 20, reps=10, spec=args.spec)
        out["config4_ik_dls_f64"] = _ik_leg(m, arm, gl, ctx, stream, spec=args.spec, dt=torch.float64)
        out["config5_fk_sdf"] = _coll_leg(ctx, stream, N, max(5, args.steps // 2), spec=args.spec, pad=args.row_pad)
        out["config5_fk_sdf"]["min_dist"]["pmc"] = _pmc_valu("pmc_coll32s.json")
        out["config5_fk_sdf"]["dists_grads"]["pmc"] = _pmc_valu("pmc_collg32s.json")
        out.update(_scene_and_coll_ik_legs(ctx, stream, N, max(5, args.steps // 2), spec=args.spec))
        out["a11_nakamura_f64"] = _nakamura_leg(m, arm, gl, ctx, stream, spec=args.spec)
        if args.spec:  # the same legs on the generic kernels (A/B of kin_plan_specialize)
            out["generic_kernels"] = {
                "config4_ik_dls": _ik_leg(m, arm, gl, ctx, stream, spec=0)["value"],
                "ik_dls_1M_targets": _ik_leg(m, arm, gl, ctx, stream, n=1 << 20, reps=3, spec=0)["value"],
                "config5_fk_sdf": {k: v["value"] for k, v in _coll_leg(ctx, stream, N, max(5, args.steps // 2),
                                                                        spec=0).items() if isinstance(v, dict)},
                # (the generic ineq_const figures include the broad phase, which both kernels have)
                "a11_nakamura_f64": _nakamura_leg(m, arm, gl, ctx, stream, spec=0)["value"]}
    if SPEC_ERRORS:
        out["specialization_errors"] = SPEC_ERRORS
    if rank == 0 and ws == 1 and not args.no_cpu:  # the CPU baseline is a single-GPU-run figure
        out["cpu_baseline"] = _cpu_baseline(m)
    sys.stdout.flush()
    os.dup2(json_fd, 1)
    os.close(json_fd)
    if rank == 0:
        print(json.dumps(out), flush=True)
    os.dup2(2, 1)  # (nothing after the line: the group's teardown may print too)
    if ctx.dist:
        ctx.dist.destroy_process_group()


if __name__ == "__main__":
    main()
