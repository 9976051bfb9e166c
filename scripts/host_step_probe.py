"""Is a small population's train step bound by the host?  Per population size:
the host time of each ``train_step`` call (enqueue only: the calls return before
the GPU finishes) against the wall time per step over a long run (one sync at
the end).  Host ~= wall means the GPU waits on the launches.

    python scripts/host_step_probe.py [--trials 2 4 64] [--steps 300]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd.population import PopulationEngine, TrialSpec, kfold_split, synthetic_mnist  # noqa: E402
from scripts.train_probe import sample_trials  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, nargs="+", default=[2, 4, 64])
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--folds", type=int, default=5)
    a = ap.parse_args()
    x, y = synthetic_mnist(60000, seed=0)
    for nt in a.trials:
        members, folds = [], []
        for t in sample_trials(nt):
            for f in range(a.folds):
                members.append(TrialSpec(t.nb_filters, t.kernel_size, t.pool_size, t.dense, t.lr, t.dropout,
                                         seed=len(members)))
                folds.append(f)
        order = torch.from_numpy(np.stack([kfold_split(60000, a.folds, f)[0] for f in folds])).cuda()
        e = PopulationEngine(members, batch=100)
        for s in range(5):
            e.train_step(x, y, order, s * 100)
        torch.cuda.synchronize()
        host = []
        t0 = time.perf_counter()
        for s in range(a.steps):
            h0 = time.perf_counter()
            e.train_step(x, y, order, (s % 400) * 100)
            host.append(time.perf_counter() - h0)
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        h = np.array(host) * 1e3
        print(f"{len(members)} members: wall {wall / a.steps * 1e3:.3f} ms/step; host per call median {np.median(h):.3f} "
              f"ms, mean {h.mean():.3f}, p90 {np.percentile(h, 90):.3f}; all calls enqueued after {t_enq:.3f} s "
              f"of {wall:.3f} s", flush=True)
        del e
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
