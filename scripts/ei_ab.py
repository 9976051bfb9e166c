"""A/B the GP scoring kernel variants in one process, interleaved.

VARIANTS: name=ENV:VAL,ENV:VAL ... on the command line (default: the occupancy
variants and the MPO_GP_DEBUG phase switches).  Each variant scores the
BASELINE configs[1] problem (1M candidates, top-5 EI) 5 times per round."""
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
KEYS = ("MPO_GP_OCC", "MPO_GP_DEBUG", "MPO_GP_DIST")
if len(sys.argv) > 1:
    VARIANTS = {}
    for arg in sys.argv[1:]:
        name, _, spec = arg.partition("=")
        VARIANTS[name] = dict(kv.split(":") for kv in spec.split(",") if kv)
else:
    VARIANTS = {"occ4": {"MPO_GP_OCC": "4"}, "occ5": {"MPO_GP_OCC": "5"}, "occ6": {"MPO_GP_OCC": "6"},
                "occ8": {"MPO_GP_OCC": "8"}, "no-mfma": {"MPO_GP_DEBUG": "1"}, "no-matern": {"MPO_GP_DEBUG": "2"},
                "no-topk": {"MPO_GP_DEBUG": "4"}, "no-mfma-matern": {"MPO_GP_DEBUG": "3"},
                "shell": {"MPO_GP_DEBUG": "7"}}
res = {b: [] for b in VARIANTS}
for rnd in range(4):
    for b in res:
        for key in KEYS:
            os.environ.pop(key, None)
        os.environ.update(VARIANTS[b])
        try:
            g.score(cand, float(y.min()), k=5)
        except Exception as e:  # a variant the library refuses (e.g. one that would spill)
            res[b].append(float("nan"))
            print(b, "refused:", str(e).splitlines()[0][:120])
            continue
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.score(cand, float(y.min()), k=5)
        e1.record()
        torch.cuda.synchronize()
        res[b].append(e0.elapsed_time(e1) / 5)
for b, v in res.items():
    print("%-16s median %.3f ms  min %.3f ms  (%.1f%% of FP64 peak)" % (b, np.median(v), np.min(v),
          100 * (200 * 201 + 200 * 42 + 30) * 1e6 / (np.median(v) * 1e-3) / 78.6e12))
