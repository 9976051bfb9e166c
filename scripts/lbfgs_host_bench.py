"""Host time of the batched L-BFGS-B driver per round (no device): a cheap numpy
objective over 3 starts, the driver's own microseconds per round."""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mod = sys.argv[1] if len(sys.argv) > 1 else "mpi_opt_amd.gp_fit"
GF = importlib.import_module(mod)

d = 5
bounds = GF.theta_bounds(d)
A = np.random.RandomState(0).randn(d + 2, d + 2)
H = A @ A.T / (d + 2) + np.eye(d + 2)


def ev(X, ids):
    X = np.asarray(X)
    v = np.einsum('bi,ij,bj->b', X - 0.3, H, X - 0.3) + 0.1 * np.sin(3 * X).sum(1)
    g = 2 * (X - 0.3) @ H + 0.3 * np.cos(3 * X)
    return v, g


rng = np.random.RandomState(1)
starts = [np.zeros(d + 2)] + [rng.uniform(bounds[:, 0], bounds[:, 1]) for _ in range(2)]
X3 = np.stack(starts)
t0 = time.perf_counter()
for _ in range(4000):
    ev(X3, [0, 1, 2])
obj = (time.perf_counter() - t0) / 4000
setulb = GF._setulb()
best = 1e9
for rep in range(7):
    t0 = time.perf_counter()
    tot = 0
    for s in range(60):
        out, rounds = GF.lbfgsb_batched(ev, starts, bounds)
        tot += rounds
    best = min(best, (time.perf_counter() - t0) / tot)
print(f"{mod}: rounds per fit {rounds}; driver us per round {(best - obj) * 1e6:.1f} (objective {obj * 1e6:.1f} us); "
      f"result {[round(o[1], 12) for o in out]}")
