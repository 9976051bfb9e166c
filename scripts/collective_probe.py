"""Cost of the pickled object collectives of the N-rank search (blocks.py
DistributedEvaluator: broadcast_object_list / all_gather_object), at the
configs[3] sizes, on a gloo group of CPU processes (no GPU):

* rank 0 broadcasts a population's 64 buffered ``ChainJob``s (the asking
  optimizer's told points, n0 = 192 at the 4th population);
* every rank all-gathers its chain results (its share of the 64 batches of 256
  points) and its (trial, fold) histories (10 epochs of loss / accuracy).

    python scripts/collective_probe.py [--ranks 8] [--reps 20]
"""
import argparse
import os
import pickle
import sys
import time

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)


def payloads(rank, ranks, n0=192, jobs=64, points=256, units=320):
    from mpi_opt_amd.models import mnist_space
    from mpi_opt_amd.optimizer import ChainJob, Optimizer

    opt = Optimizer(mnist_space(), base_estimator="dummy", random_state=0)
    X = opt.ask(n0)
    opt.tell(X, list(np.random.default_rng(0).random(n0)))
    chain_jobs = [ChainJob(opt, seed=i, n_points=points, strategy="cl_min") for i in range(jobs)]
    mine = [X[:points] for _ in range(jobs // ranks)]               # this rank's batches of points
    hist = [{"loss": list(np.random.default_rng(u).random(10)), "val_loss": list(np.random.default_rng(u + 1).random(10)),
             "acc": list(np.random.default_rng(u + 2).random(10)),
             "val_acc": list(np.random.default_rng(u + 3).random(10))} for u in range(units // ranks)]
    return chain_jobs, (mine, hist)


def worker(rank, ranks, reps, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ranks)
    jobs, gathered = payloads(rank, ranks)
    res = {}
    for name in ("broadcast", "all_gather"):
        times = []
        for r in range(reps + 2):
            dist.barrier()
            t0 = time.perf_counter()
            if name == "broadcast":
                box = [jobs if rank == 0 else None]
                dist.broadcast_object_list(box, src=0)
            else:
                lst = [None] * ranks
                dist.all_gather_object(lst, gathered)
            dt = time.perf_counter() - t0
            if r >= 2:
                times.append(dt)
        t = torch.tensor([float(np.median(times))], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        res[name] = float(t.item())
    if rank == 0:
        res["broadcast_bytes"] = len(pickle.dumps(jobs))
        res["all_gather_bytes_per_rank"] = len(pickle.dumps(gathered))
        out.put(res)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--port", type=int, default=29613)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, a.ranks, a.reps, a.port, q)) for r in range(a.ranks)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
    print(f"{a.ranks} gloo ranks (CPU), median of {a.reps}, max over ranks:")
    print(f"  broadcast_object_list of 64 ChainJobs (n0 = 192): {res['broadcast'] * 1e3:.2f} ms, "
          f"{res['broadcast_bytes'] / 1e3:.1f} kB pickled")
    print(f"  all_gather_object of chain points + histories: {res['all_gather'] * 1e3:.2f} ms, "
          f"{res['all_gather_bytes_per_rank'] / 1e3:.1f} kB per rank")


if __name__ == "__main__":
    main()
