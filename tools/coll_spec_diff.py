"""Specialised vs generic k_coll (fp32) on the 64-box scene of tests/test_collision.py::
test_gpu_collision_lds_box_limit: counts and sizes of differing entries."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("kinematics.jl_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import kinhip  # noqa: E402
import oracle as O  # noqa: E402
from test_collision import _T, _gpu_setup  # noqa: E402

dev = torch.device("cuda", 0)
for n_boxes in (64, 65):
    m, sscc, arm = _gpu_setup(False)
    rng = np.random.default_rng(100 + n_boxes)
    poses, widths = [], []
    for _ in range(n_boxes):
        R = O.rpy_to_matrix(rng.uniform(-np.pi, np.pi, 3)) if rng.random() < 0.5 else np.eye(3)
        poses.append(_T(rng.uniform([-1, -1, 0], [1.5, 1, 1.5]), R))
        widths.append(rng.uniform(0.02, 0.2, 3))
    sdf = kinhip.UnionSDF([kinhip.BoxSDF(P, w) for P, w in zip(poses, widths)])
    Q = torch.tensor(rng.uniform(-1.2, 1.2, (8, 2000)), dtype=torch.float32, device=dev)
    gen = sscc.plan(arm, dtype=torch.float32)
    spe = sscc.plan(arm, dtype=torch.float32).specialize()
    D0, G0, M0 = gen.run(sdf, Q, grads=True, min_dist=True)
    D1, G1, M1 = spe.run(sdf, Q, grads=True, min_dist=True)
    d = (G0 - G1).abs()
    nz = torch.nonzero(d > 0)
    print(n_boxes, "D equal", torch.equal(D0, D1), "G diff entries", int((d > 0).sum()), "max", float(d.max()),
          "first", nz[:5].tolist(), [(float(G0[tuple(i)]), float(G1[tuple(i)])) for i in nz[:5].tolist()])
