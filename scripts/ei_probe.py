"""Run the GP scoring kernel a few times (for PMC passes)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd import synthetic  # noqa: E402
from mpi_opt_amd.gp import DeviceGP  # noqa: E402

X, y = synthetic.gp_problem(200, 10, 0)
ls = np.array([16.2, 1.91, 1.65, 9.84, 1.84, 2.94, 2.45, 9.09, 8.13, 1.94])
g = DeviceGP(X, y, 17.4955, ls, 0.0465)
cand = torch.from_numpy(synthetic.gp_candidates(1_000_000, 10, seed=1)).cuda()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    g.score(cand, float(y.min()), k=5)
torch.cuda.synchronize()
print("done")
