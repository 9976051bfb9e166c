"""Throughput of concurrent cl_min chains on one GPU (the configs[3] search's
optimizer term): an optimizer told n points of a synthetic objective in the mnist
space, then ``jobs`` ask(k) batches (ChainJob) run on T worker threads; reports
refits per second for each T.  ``--driver scipy`` runs the refits and polishes
with scipy's setulb driven from Python instead of libmpo.so's host L-BFGS-B.
Also the single-thread refit latency."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd import gp_fit as GF  # noqa: E402
from mpi_opt_amd import optimizer as O  # noqa: E402
from mpi_opt_amd.chains import ThreadChainExecutor  # noqa: E402
from mpi_opt_amd.models import mnist_space  # noqa: E402
from mpi_opt_amd.space import Space  # noqa: E402


def objective(x):
    nb, pool, ks, dense, drop = x
    return float(((nb - 30) / 40) ** 2 + ((pool - 4) / 8) ** 2 + ((ks - 5) / 8) ** 2 + ((dense - 120) / 150) ** 2
                 + (drop - 0.3) ** 2 + 0.05 * np.sin(nb * dense / 300.0))


def batcher_stats():
    import ctypes

    from mpi_opt_amd import _lib

    la, ro = ctypes.c_int64(), ctypes.c_int64()
    _lib.check(_lib.lib().mpo_gp_lml_batcher_stats(_lib.lml_batcher(0), ctypes.byref(la), ctypes.byref(ro)))
    return la.value, ro.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=96)
    ap.add_argument("--k", type=int, default=8, help="points per ask batch")
    ap.add_argument("--jobs", type=int, default=32)
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 4, 8])
    ap.add_argument("--driver", choices=["native", "scipy"], default="native")
    a = ap.parse_args()
    if a.driver == "scipy":
        fit0, pol0 = GF.fit_lml, O.polish_lockstep
        O.fit_lml = lambda *args, **kw: fit0(*args, driver="scipy", **kw)
        O.polish_lockstep = lambda *args, **kw: pol0(*args, driver="scipy", **kw)
    if os.environ.get("PY_SWITCH"):
        sys.setswitchinterval(float(os.environ["PY_SWITCH"]))
    print("switch interval", sys.getswitchinterval())
    dev = torch.device("cuda:0")
    space = Space(mnist_space())
    rng = np.random.RandomState(0)
    pts = space.rvs(n_samples=a.n, random_state=rng)
    ys = [objective(p) for p in pts]
    opt = O.Optimizer(mnist_space(), random_state=1, device=dev)
    opt.tell(pts[:-1], ys[:-1], fit=False)
    opt.tell(pts[-1], ys[-1])
    # single-thread refit latency
    Xt = space.transform(pts)
    t0 = time.perf_counter()
    for s in range(5):
        _, det = GF.fit_lml(Xt, np.asarray(ys), random_state=s, device=dev, return_details=True, driver=a.driver)
    torch.cuda.synchronize()
    print(f"driver={a.driver} n={a.n}: one refit {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms "
          f"({det['launches']} rounds)", flush=True)
    for T in a.threads:
        ex = ThreadChainExecutor(dev, workers=T)
        jobs = [O.ChainJob(opt, 1000 + j, a.k, "cl_min") for j in range(a.jobs)]
        # warm: one job per worker (graph capture, stream setup)
        ex.run_now(jobs[:T])
        O.reset_stats()
        t0 = time.perf_counter()
        la0, ro0 = batcher_stats()
        ex.run_now(jobs)
        dt = time.perf_counter() - t0
        la1, ro1 = batcher_stats()
        st = dict(O.STATS)
        ex.close()
        print(f"  threads {T}: {st['refits']} refits in {dt:.2f} s = {st['refits'] / dt:.1f} refits/s; per refit "
              f"fit {st['refit_s'] / st['refits'] * 1e3:.2f} ms, proposal {st['propose_s'] / st['refits'] * 1e3:.2f} ms "
              f"(polish {st['polish_s'] / st['refits'] * 1e3:.2f}); {ro1 - ro0} LML rounds in {la1 - la0} grouped launch sets",
              flush=True)


if __name__ == "__main__":
    main()
