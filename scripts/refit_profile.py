"""Host-side profile of the cl_min chain (what holds the GIL): cProfile of one
ask(k) ChainJob at n told points, single thread, top functions by own time."""
import cProfile
import os
import pstats
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd import optimizer as O  # noqa: E402
from mpi_opt_amd.models import mnist_space  # noqa: E402
from mpi_opt_amd.space import Space  # noqa: E402
from scripts.chain_probe import objective  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 96
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda:0")
space = Space(mnist_space())
pts = space.rvs(n_samples=n, random_state=np.random.RandomState(0))
ys = [objective(p) for p in pts]
opt = O.Optimizer(mnist_space(), random_state=1, device=dev)
opt.tell(pts[:-1], ys[:-1], fit=False)
opt.tell(pts[-1], ys[-1])
O.ChainJob(opt, 7, 2, "cl_min").run(dev)   # warm
job = O.ChainJob(opt, 11, k, "cl_min")
pr = cProfile.Profile()
import time
t0, c0 = time.perf_counter(), time.thread_time()
pr.enable()
job.run(dev)
pr.disable()
wall, cpu = time.perf_counter() - t0, time.thread_time() - c0
print(f"n={n} ask({k}): {wall * 1e3:.1f} ms wall, {cpu * 1e3:.1f} ms thread CPU, {(k + 1)} refits")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(28)
