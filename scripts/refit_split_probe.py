"""Where one refit's time goes outside its L-BFGS-B rounds: DeviceLML
construction (device copies of X, y; workspace, pinned round buffers) vs the
fit call itself, at n observations (d = 5), single thread."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_opt_amd import gp_fit as GF  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 96
    d = 5
    rng = np.random.RandomState(0)
    X = rng.rand(n, d)
    y = np.sin(X @ rng.randn(d)) + 0.1 * rng.randn(n)
    yn, _, _ = GF.normalize_targets(y)
    bounds = GF.theta_bounds(d)
    starts = np.array([np.zeros(d + 2)] + [rng.uniform(bounds[:, 0], bounds[:, 1]) for _ in range(2)])
    dev = torch.device("cuda:0")
    for _ in range(3):
        GF.DeviceLML(X, yn, device=dev).fit(starts, bounds)
    torch.cuda.synchronize()
    tc = tf = 0.0
    rounds = 0
    R = 20
    for _ in range(R):
        t0 = time.perf_counter()
        lml = GF.DeviceLML(X, yn, device=dev)
        lml._ensure(3)
        t1 = time.perf_counter()
        _, r = lml.fit(starts, bounds)
        t2 = time.perf_counter()
        tc += t1 - t0
        tf += t2 - t1
        rounds += r
    print(f"n={n}: construct {tc / R * 1e3:.3f} ms, fit {tf / R * 1e3:.3f} ms ({rounds / R:.0f} rounds, "
          f"{tf / rounds * 1e6:.1f} us per round)", flush=True)


if __name__ == "__main__":
    main()
