"""A/B the GP scoring kernel variants (candidates per workgroup / occupancy) in one process, interleaved."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_opt_amd import synthetic  # noqa: E402
from mpi_opt_amd.gp import DeviceGP  # noqa: E402

X, y = synthetic.gp_problem(200, 10, 0)
ls = np.array([16.2, 1.91, 1.65, 9.84, 1.84, 2.94, 2.45, 9.09, 8.13, 1.94])
g = DeviceGP(X, y, 17.4955, ls, 0.0465)
cand = torch.from_numpy(synthetic.gp_candidates(1_000_000, 10, seed=1)).cuda()
VARIANTS = {"bm16/occ5": {"MPO_GP_BM": "16", "MPO_GP_OCC": "5"},
            "bm16/occ6": {"MPO_GP_BM": "16", "MPO_GP_OCC": "6"},
            "bm16/occ8": {"MPO_GP_BM": "16", "MPO_GP_OCC": "8"}}
res = {b: [] for b in VARIANTS}
for rnd in range(4):
    for b in res:
        os.environ.update(VARIANTS[b])
        g.score(cand, float(y.min()), k=0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.score(cand, float(y.min()), k=0)
        e1.record()
        torch.cuda.synchronize()
        res[b].append(e0.elapsed_time(e1) / 5)
for b, v in res.items():
    print("%-10s median %.3f ms  min %.3f ms  (%.1f%% of FP64 peak)" % (b, np.median(v), np.min(v),
          100 * (200 * 201 + 200 * 42 + 30) * 1e6 / (np.median(v) * 1e-3) / 78.6e12))
