"""A/B the GP scoring variants (candidates per workgroup) in one process, interleaved."""
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
res = {b: [] for b in ("32/1", "16/5", "16/6")}
for rnd in range(4):
    for b in res:
        os.environ["MPO_GP_BM"], os.environ["MPO_GP_OCC"] = b.split("/")
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
    print("BM/occ=%s  median %.3f ms  min %.3f ms" % (b, np.median(v), np.min(v)))
