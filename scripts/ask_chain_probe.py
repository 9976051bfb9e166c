"""A lone cl_min chain: bench.py's ask256 leg (256 tells, then ask(N) on one
thread, every refit at n = 256 .. 256 + N) with a shorter batch by default, plus
the LML rounds the native L-BFGS-B driver ran per refit (DeviceLML.fit).

    python scripts/ask_chain_probe.py [--ask-n 64] [--reps 2]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd import gp_fit as GF  # noqa: E402
from mpi_opt_amd import optimizer as OPT  # noqa: E402
from mpi_opt_amd.models import mnist_space  # noqa: E402

ROUNDS = [0]
_fit = GF.DeviceLML.fit


def _counting_fit(self, *a, **k):
    res, rounds = _fit(self, *a, **k)
    ROUNDS[0] += rounds
    return res, rounds


GF.DeviceLML.fit = _counting_fit


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ask-n", type=int, default=64)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    for rep in range(a.reps):
        rng = np.random.RandomState(256)
        opt = OPT.Optimizer(mnist_space(), random_state=13579, device="cuda:0")
        pts = opt.space.rvs(n_samples=256, random_state=rng)
        ys = [float(((p[0] - 30) / 40) ** 2 + ((p[3] - 120) / 150) ** 2 + (p[4] - 0.3) ** 2 + 0.1 * rng.rand())
              for p in pts]
        opt.tell(pts[:-1], ys[:-1], fit=False)
        opt.tell(pts[-1], ys[-1])
        OPT.reset_stats()
        ROUNDS[0] = 0
        t0 = time.perf_counter()
        batch = opt.ask(a.ask_n)
        dt = time.perf_counter() - t0
        st = dict(OPT.STATS)
        print(f"rep {rep}: ask({a.ask_n}) {dt:.3f} s, {st['refits']} refits, "
              f"{1e3 * st['refit_s'] / st['refits']:.2f} ms/refit, {1e3 * st['propose_s'] / st['refits']:.2f} ms/proposal, "
              f"{ROUNDS[0] / st['refits']:.1f} LML rounds/refit ({1e6 * st['refit_s'] / max(1, ROUNDS[0]):.0f} us/round), "
              f"first point {list(batch[0])}", flush=True)


if __name__ == "__main__":
    main()
