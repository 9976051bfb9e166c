"""Cost of the N-rank search's rounds (blocks.DistributedEvaluator, fixed-layout
tensor collectives since r06) at the configs[3] sizes, on a gloo group of CPU
processes (no GPU; the training and the chains are stubs that return at once):

* a chains round: rank 0's 64 buffered ``ChainJob``s (n0 = 192 told points, 256
  points each) encoded and broadcast, LPT-dealt, every rank's batches, refit
  accounts and error text all-gathered;
* a train round: 64 trials x 5 folds, LPT-sharded, 10-epoch histories all-gathered.

    python scripts/tensor_collective_probe.py [--ranks 8] [--reps 20]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Runner:
    def __init__(self, X):
        self.X = X

    def run_now(self, jobs):
        return [(self.X[:j.n_points], None) for j in jobs]


class _Local:
    device = None

    def units(self, params_list):
        return [(t, f, None, 1.0 + t % 7) for t in range(len(params_list)) for f in range(5)]

    def train_units(self, units, seed_base=0, trial_ids=None):
        rng = np.random.default_rng(seed_base)
        return {(t, f): {"val_loss": list(rng.random(10)), "val_acc": list(rng.random(10))} for (t, f, _, _) in units}

    def foms(self, params_list, results):
        return [float(np.mean([results[(t, f)]["val_loss"][-1] for f in range(5)])) for t in range(len(params_list))]


def worker(rank, ranks, reps, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ranks)
    from mpi_opt_amd.blocks import DistributedEvaluator
    from mpi_opt_amd.models import mnist_space
    from mpi_opt_amd.optimizer import ChainJob, Optimizer

    opt = Optimizer(mnist_space(), base_estimator="dummy", random_state=0)
    X = opt.ask(192)
    opt.tell(X, list(np.random.default_rng(0).random(192)))
    pts = opt.space.rvs(n_samples=256, random_state=np.random.RandomState(1))
    ev = DistributedEvaluator(_Local(), chain_runner=_Runner([list(p) for p in pts]))
    res = {}
    if rank == 0:
        jobs = [ChainJob(opt, seed=i, n_points=256, strategy="cl_min") for i in range(64)]
        params = [list(p) for p in pts[:64]]
        for name, fn in (("chains", lambda: ev.chains(jobs)), ("train", lambda: ev.evaluate(params))):
            times = []
            for r in range(reps + 2):
                t0 = time.perf_counter()
                fn()
                if r >= 2:
                    times.append(time.perf_counter() - t0)
            res[name] = float(np.median(times))
        ev.shutdown()
        res["config_broadcasts"] = ev.config_broadcasts
        out.put(res)
    else:
        ev.serve()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--port", type=int, default=29623)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, a.ranks, a.reps, a.port, q)) for r in range(a.ranks)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
    print(f"{a.ranks} gloo ranks (CPU), median of {a.reps} rounds on rank 0 (tensor collectives, r06):")
    print(f"  chains round, 64 ChainJobs (n0 = 192, 256 points each): {res['chains'] * 1e3:.2f} ms "
          f"(config object broadcast {res['config_broadcasts']}x, first round only)")
    print(f"  train round, 64 trials x 5 folds, 10-epoch histories: {res['train'] * 1e3:.2f} ms")


if __name__ == "__main__":
    main()
