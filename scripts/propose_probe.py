"""Where one proposal's time goes (Optimizer._fit_and_propose after the refit):
mpo_gp_prepare (DeviceGP construction), the 10 000-candidate scoring, and the
3 x 5 L-BFGS-B polish (rounds x one mpo_gp_acq_grad launch)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd import gp_fit as GF  # noqa: E402
from mpi_opt_amd import optimizer as OPT  # noqa: E402
from mpi_opt_amd.gp import DeviceGP  # noqa: E402

dev = torch.device("cuda:0")
d = 5
for n in (64, 128, 256, 512):
    rng = np.random.RandomState(n)
    X = rng.uniform(size=(n, d))
    y = np.sin(X @ rng.uniform(-2, 2, d)) + 0.1 * rng.randn(n)
    amp, ls, noise = 1.3, rng.uniform(0.3, 3.0, d), 1e-3
    DeviceGP(X, y, amp, ls, noise, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        g = DeviceGP(X, y, amp, ls, noise, device=dev)
    torch.cuda.synchronize()
    t_prep = (time.perf_counter() - t0) / 3
    C = rng.uniform(size=(10000, d))
    g.score(C, float(y.min()), acqs=("EI", "LCB", "PI"), k=5, want_mu_sd=False, want_values=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        sc = g.score(C, float(y.min()), acqs=("EI", "LCB", "PI"), k=5, want_mu_sd=False, want_values=False)
        [sc["topk"][a][0].cpu() for a in ("EI", "LCB", "PI")]
    t_score = (time.perf_counter() - t0) / 5
    P = rng.uniform(size=(15, d))
    codes = [1, 4, 2] * 5
    g.acq_grad(P, codes, float(y.min()))
    t0 = time.perf_counter()
    for _ in range(20):
        g.acq_grad(P, codes, float(y.min()))
    t_ag = (time.perf_counter() - t0) / 20
    model = OPT.GPModel(X, y, amp, ls, noise, device=dev)
    model._dev = g
    starts = [C[i] for i in range(15)]
    acqs = ["EI"] * 5 + ["LCB"] * 5 + ["PI"] * 5
    rounds = {}

    def ev(Xb, ids, _g=g, _codes=np.array([OPT._lib.ACQ_FLAGS[a] for a in acqs])):
        rounds["n"] = rounds.get("n", 0) + 1
        return _g.acq_grad(Xb, _codes[ids], float(y.min()), 0.01, 1.96)

    t0 = time.perf_counter()
    GF.lbfgsb_batched(ev, starts, [(0.0, 1.0)] * d, ftol=GF.FMIN_FTOL, maxiter=20)
    t_pol = time.perf_counter() - t0
    print(f"n={n:4d}: prepare {t_prep * 1e3:7.2f} ms | score 10k x3 {t_score * 1e3:6.2f} ms | acq_grad(15) "
          f"round trip {t_ag * 1e6:7.1f} us | polish {t_pol * 1e3:7.2f} ms in {rounds['n']} rounds", flush=True)
