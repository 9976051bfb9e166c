"""Time one skopt-style refit + proposal (Optimizer._fit_and_propose) at several
numbers of observations n, split into the GP refit, the candidate scoring and the
acquisition polish (3 x 5 lockstep L-BFGS-B runs on mpo_gp_acq_grad)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd import optimizer as OPT  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[50, 200, 256, 500])
ap.add_argument("--d", type=int, default=10)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()

timers = {}


def timed(name, fn):
    def w(*args, **kw):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*args, **kw)
        torch.cuda.synchronize()
        timers[name] = timers.get(name, 0.0) + time.perf_counter() - t0
        return r
    return w


OPT.fit_gp_hyperparameters = timed("refit", OPT.fit_gp_hyperparameters)
OPT.polish_lockstep = timed("polish", OPT.polish_lockstep)
OPT.Optimizer._score_topk = timed("score", OPT.Optimizer._score_topk)
OPT.GPModel.predict_mean = timed("prepare+predict", OPT.GPModel.predict_mean)
OPT.Space.rvs = timed("rvs", OPT.Space.rvs)
OPT.Space.transform = timed("transform", OPT.Space.transform)

for n in a.n:
    rng = np.random.RandomState(n)
    dims = [(0.0, 1.0)] * a.d
    X = rng.uniform(size=(n, a.d))
    y = np.sin(X @ rng.uniform(-2, 2, a.d)) + 0.1 * rng.randn(n)
    opt = OPT.Optimizer(dims, random_state=1, device="cuda:0")
    opt.tell(X[:-1].tolist(), y[:-1].tolist(), fit=False)
    for r in range(a.reps):
        timers.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        opt._tell(X[-1].tolist(), float(y[-1]))      # one refit + proposal at n observations
        total = time.perf_counter() - t0
        opt.Xi.pop()
        opt.yi.pop()
        opt._n_initial_points += 1
    print(f"n={n} d={a.d}: tell {total * 1e3:.1f} ms = refit {timers['refit'] * 1e3:.1f} + score "
          f"{timers['score'] * 1e3:.1f} + polish {timers['polish'] * 1e3:.1f} ms; " +
          ", ".join(f"{k} {v * 1e3:.1f}" for k, v in timers.items()), flush=True)
