"""Where a GP refit's time goes at the search's sizes (mnist space, d = 5).

For each n: one skopt refit (fit_lml: 3 L-BFGS-B starts in lockstep) split into
the number of lockstep rounds (= LML launches), the device time per launch (HIP
events around mpo_gp_lml_grad alone) and the round-trip time of one
DeviceLML.evaluate (host staging + launch + synchronising copy); then one
refit + proposal (Optimizer._tell) split as scripts/ask_probe.py does; then,
optionally, a cl_min batch ask(k) after n tells.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd import _lib  # noqa: E402
from mpi_opt_amd import gp_fit as GF  # noqa: E402
from mpi_opt_amd import optimizer as OPT  # noqa: E402
from mpi_opt_amd.models import mnist_space  # noqa: E402
from mpi_opt_amd.space import Space  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[16, 64, 128, 256, 512])
ap.add_argument("--ask", type=int, default=0, help="also time ask(k) after the largest n tells")
a = ap.parse_args()

dev = torch.device("cuda:0")
space = Space(mnist_space())


def objective(x):
    nb, pool, ks, dense, drop = x
    return float(((nb - 30) / 40) ** 2 + ((pool - 4) / 8) ** 2 + ((ks - 5) / 8) ** 2 + ((dense - 120) / 150) ** 2
                 + (drop - 0.3) ** 2 + 0.05 * np.sin(nb * dense / 300.0))


for n in a.n:
    rng = np.random.RandomState(n)
    pts = space.rvs(n_samples=n, random_state=rng)
    y = np.array([objective(p) for p in pts])
    Xt = space.transform(pts)
    yn, _, _ = GF.normalize_targets(y)
    lml = GF.DeviceLML(Xt, yn, device=dev)
    thetas = np.zeros((3, Xt.shape[1] + 2))
    lml.evaluate(thetas)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 50
    for _ in range(reps):
        lml.evaluate(thetas)
    rt = (time.perf_counter() - t0) / reps
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.current_stream(dev)
    e0.record(s)
    for _ in range(reps):
        _lib.check(_lib.lib().mpo_gp_lml_grad(
            _lib.ptr(lml.X), _lib.ptr(lml.y), lml.n, lml.d, _lib.ptr(lml.theta_d), 3, _lib.ptr(lml.lml_d),
            _lib.ptr(lml.grad_d), _lib.ptr(lml.info_d), _lib.ptr(lml.ws), lml.ws_bytes, s.cuda_stream), "lml")
    e1.record(s)
    e1.synchronize()
    kt = e0.elapsed_time(e1) / reps / 1e3
    t0 = time.perf_counter()
    _, det = GF.fit_lml(Xt, y, random_state=7, device=dev, return_details=True)
    fit = time.perf_counter() - t0
    L = det["launches"]
    print(f"n={n:4d}: refit {fit * 1e3:7.1f} ms = {L} rounds x {fit / L * 1e6:6.1f} us; one evaluate round trip "
          f"{rt * 1e6:6.1f} us, device {kt * 1e6:6.1f} us per launch -> host share "
          f"{(fit / L - kt) * 1e6:6.1f} us/round", flush=True)

    opt = OPT.Optimizer(mnist_space(), random_state=1, device=dev)
    opt.tell(pts[:-1], list(y[:-1]), fit=False)
    t0 = time.perf_counter()
    opt.tell(pts[-1], float(y[-1]))
    torch.cuda.synchronize()
    print(f"        refit + proposal (one tell): {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)

if a.ask:
    t0 = time.perf_counter()
    batch = opt.ask(a.ask)
    dt = time.perf_counter() - t0
    print(f"ask({a.ask}) after {a.n[-1]} tells: {dt:.2f} s = {dt / (a.ask + 1) * 1e3:.1f} ms per refit+proposal "
          f"({a.ask + 1} refits)", flush=True)
