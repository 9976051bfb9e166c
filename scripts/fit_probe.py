"""Time the device GP refit (n obs, d dims) and the host sklearn refit it replaces."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_opt_amd import synthetic  # noqa: E402
from mpi_opt_amd.gp_fit import DeviceLML, fit_lml, normalize_targets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=200)
ap.add_argument("--d", type=int, default=10)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
X, y = synthetic.gp_problem(a.n, a.d, 0)
for r in range(a.reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, det = fit_lml(X, y, random_state=0, device="cuda:0", return_details=True)
    dt = time.perf_counter() - t0
    print(f"fit n={a.n} d={a.d}: {dt * 1e3:.1f} ms, {det['launches']} launches, "
          f"{dt / det['launches'] * 1e3:.2f} ms/launch, lml {det['lml']:.9f}", flush=True)
dev = DeviceLML(X, normalize_targets(y)[0], device="cuda:0")
T = np.zeros((3, a.d + 2))
dev.evaluate(T)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    dev.evaluate(T)
print(f"evaluate(B=3) round trip {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms", flush=True)
