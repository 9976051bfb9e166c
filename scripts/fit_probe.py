"""Time the device GP refit at several n: the LML kernel alone (HIP events, B=3
thetas per launch, the three L-BFGS-B starts) and a whole skopt refit
(launches x per-launch + the host L-BFGS-B).  --kernels picks the LML
kernels compared (MPO_FIT_KERNEL): panel (LDS Cholesky, n <= 200), split
(multi-workgroup block sweep)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd import _lib, synthetic  # noqa: E402
from mpi_opt_amd.gp_fit import DeviceLML, fit_lml, normalize_targets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[200, 256, 500])
ap.add_argument("--d", type=int, default=10)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--kernels", nargs="+", default=["split", "panel"])
ap.add_argument("--phases", action="store_true", help="kernel time up to each MPO_FIT_DEBUG stop (1 K, 2 factor, 4 alpha)")
a = ap.parse_args()


def kernel_ms(dev, T, reps=20):
    dev.evaluate(T)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        _lib.check(_lib.lib().mpo_gp_lml_grad(
            _lib.ptr(dev.X), _lib.ptr(dev.y), dev.n, dev.d, _lib.ptr(dev.theta_d), T.shape[0], _lib.ptr(dev.lml_d),
            _lib.ptr(dev.grad_d), _lib.ptr(dev.info_d), _lib.ptr(dev.ws), dev.ws_bytes, s.cuda_stream))
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for n in a.n:
    X, y = synthetic.gp_problem(n, a.d, 0)
    for kern in a.kernels:
        if kern == "panel" and n > 200:
            continue
        os.environ["MPO_FIT_KERNEL"] = kern   # panel | split
        dev = DeviceLML(X, normalize_targets(y)[0], device="cuda:0")
        T = np.zeros((3, a.d + 2))
        T[1] += 0.5
        T[2] -= 0.5
        k_ms = kernel_ms(dev, T)
        if a.phases:
            ph = {}
            for stop in ("1", "2", "4", "6", "7"):
                os.environ["MPO_FIT_DEBUG"] = stop
                ph[stop] = kernel_ms(dev, T)
            os.environ.pop("MPO_FIT_DEBUG")
            print(f"n={n} kernel={kern} phases (cumulative ms): K {ph['1']:.3f}, factor {ph['2']:.3f}, "
                  f"alpha {ph['4']:.3f}, all {k_ms:.3f}; without pivot sweeps {ph['6']:.3f}, without "
                  f"trailing updates {ph['7']:.3f}", flush=True)
        for r in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, det = fit_lml(X, y, random_state=0, device="cuda:0", return_details=True)
            dt = time.perf_counter() - t0
        if a.reps == 0:
            print(f"n={n} d={a.d} kernel={kern}: {k_ms:.3f} ms per launch (3 thetas)", flush=True)
            continue
        print(f"n={n} d={a.d} kernel={kern}: {k_ms:.3f} ms per launch (3 thetas); refit {dt * 1e3:.1f} ms, "
              f"{det['launches']} launches ({dt / det['launches'] * 1e3:.2f} ms/launch with host), "
              f"lml {det['lml']:.9f}", flush=True)
