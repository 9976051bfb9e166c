"""One LML round (DeviceLML.evaluate of 3 thetas) repeated at one n, for a
kernel trace: wall time per round on one thread, to set against the summed
kernel durations and the gaps between the round's launches (rocprofv3
--kernel-trace; scripts/lml_round_gaps.py reads the trace)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd import gp_fit as GF  # noqa: E402


def main():
    ns = [int(v) for v in sys.argv[1:]] or [96]
    d = 5
    for n in ns:
        rng = np.random.RandomState(0)
        X = rng.rand(n, d)
        y = np.sin(X @ rng.randn(d))
        yn, _, _ = GF.normalize_targets(y)
        th = np.zeros((3, d + 2))
        lml = GF.DeviceLML(X, yn, device="cuda:0")
        for _ in range(20):
            lml.evaluate(th)
        torch.cuda.synchronize()
        R = 300
        t0 = time.perf_counter()
        for _ in range(R):
            lml.evaluate(th)
        dt = (time.perf_counter() - t0) / R
        print(f"n={n}: {dt * 1e6:.1f} us per round (wall, 1 thread)", flush=True)


if __name__ == "__main__":
    main()
