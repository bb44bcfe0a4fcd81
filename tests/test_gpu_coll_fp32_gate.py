"""fp32 collision parity on the bench's exact path: config 5's dataset (2^20 Fetch
configurations, seed 555, bench.py coll_shard), the fridge scene (door 2.0 rad, base (1.2, 0, 0)), the 14
build-defined arm spheres, the plan-specialised kernels with the hardware sin/cos -- min-distance, and
distances + 14x8 gradients in the plain and the tiled (tile 8192) layouts -- against the oracle evaluated
at the fp32-rounded angles (src/sdf.jl, src/collision.jl:67-94 restated).

  * distances and minimum distance: 1e-6 absolute, the north star's bound (measured 5.2e-7 / 4.1e-7,
    tools/coll_fp32_err.py, profiles/r03_coll_fp32_err.txt);
  * tiled == plain, bit for bit;
  * gradients vs the reference's forward difference (eps 1e-7): |g - g_ref| <= 5e-6 (1 + 1 / rho), rho
    = |sdf(centre)|.  Derivation: the fp32 sphere centre is off by delta <= ~1e-6 (chain rounding + the
    hardware trig, the distance bound above) and J3 entries by ~1e-6; the box normal at an edge or
    corner turns by delta / rho, so |dg| <= |J3| delta / rho + |n| dJ with |J3| <= ~1.5 m; the forward
    difference of the reference adds ~eps |d''| <= 1e-7 (1 + 1 / rho).  Every entry beyond the bound must
    sit at a kink of the distance (argmin switch between boxes, edge / corner region), proven by the
    oracle's one-sided differences, be an entry where the reference's own forward difference is the
    inaccurate one (edge curvature; the GPU matches the central difference), or be an argmin near-tie:
    another box within 2e-6 (twice the distance bound) of the minimum whose own gradient the GPU returns
    (tests/test_collision.py::_assert_mismatches_at_kinks)."""
import os
import sys

import numpy as np
import pytest
import torch

import oracle as O
from conftest import ROOT, golden

sys.path.insert(0, ROOT)
import kinhip  # noqa: E402
from test_collision import _assert_mismatches_at_kinks  # noqa: E402

pytestmark = pytest.mark.gpu

TOL = 1e-6


def test_coll_fp32_bench_path_at_the_north_star_bound():
    from bench import fridge_scene
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dev = torch.device("cuda", 0)
    m, arm, sscc, sdf = fridge_scene()
    n = 1 << 20
    Q = kinhip.uniform_configs([j.lower_limit for j in arm], [j.upper_limit for j in arm], n, start=0, seed=555,
                               dtype=torch.float32, device=dev)  # bench.py coll_shard, rank 0
    plan = sscc.plan(arm, dtype=torch.float32).specialize()
    assert plan.specialized == kinhip.KIN_SPEC_COLL
    _, _, Mn = plan.run(sdf, Q, dists=False, min_dist=True)
    D, G, Mn2 = plan.run(sdf, Q, grads=True, min_dist=True)
    # the bench's exact layout: rows padded to ld = n + 256 (bench.py _coll_leg), equal bit for bit
    ld = n + 256
    Qb = torch.zeros((8, ld), dtype=torch.float32, device=dev)
    Qb[:, :n] = Q
    Dp = torch.zeros((plan.n_sph, ld), dtype=torch.float32, device=dev)[:, :n]
    Gp = torch.zeros((plan.n_sph, 8, ld), dtype=torch.float32, device=dev)[:, :, :n]
    plan.run(sdf, Qb[:, :n], dists=Dp, grads=Gp)
    torch.cuda.synchronize()
    assert torch.equal(Dp, D) and torch.equal(Gp, G)
    tree = O.parse_urdf_tree(golden("fetch.urdf"))
    om = O.OracleMech(tree)
    sph, rad = [], []
    for name, c, r in kinhip.FETCH_ARM_SPHERES:
        T = np.eye(4)
        T[:3, 3] = c
        sph.append(om.add_new_link(tree.link_id(name), T))
        rad.append(r)
    poses, widths = O.fridge_boxes(O.parse_urdf_tree(golden("fridge.urdf")))
    box = O.OracleUnionSDF(poses, widths)
    ids = [tree.joint_id(x) for x in kinhip.FETCH_ARM_JOINTS]
    q = Q.double().cpu().numpy()
    rd, rg = O.coll_batch(om, box, q, ids, sph, rad, n_threads=16)
    d = D.double().cpu().numpy()
    ed = np.abs(d - rd).max()
    em = max(np.abs(Mn.double().cpu().numpy() - rd.min(0)).max(), np.abs(Mn2.double().cpu().numpy() - rd.min(0)).max())
    print(f"fp32 bench path 2^20: max |dist - oracle| {ed:.3e}, max |min_dist - oracle| {em:.3e}")
    assert ed <= TOL and em <= TOL
    rho = np.abs(rd + np.asarray(rad)[:, None])
    gtol = 5e-6 * (1.0 + 1.0 / np.maximum(rho, 1e-12))[:, None, :]
    nk = _assert_mismatches_at_kinks(om, box, q, ids, sph, rad, G.double().cpu().numpy(), rg, gtol, h=1e-5,
                                     boxes=(poses, widths), dtie=2 * TOL)
    print(f"gradient entries beyond 5e-6 (1 + 1/rho), all at kinks: {nk} of {G.numel()}")
