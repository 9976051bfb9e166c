"""bench.py's train-leg shard ratio (one GPU's LPT share of the 320-member
population against the whole population, same process) measured in three
orders -- full then share (as bench.py), share then full, and interleaved
windows -- to see whether the order of the two timings moves the ratio."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import sample_trials  # noqa: E402
from mpi_opt_amd.blocks import lpt_assign  # noqa: E402
from mpi_opt_amd.population import PopulationEngine, TrialSpec, kfold_split, synthetic_mnist  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    members = []
    for t in sample_trials(64, seed=13579):
        for f in range(5):
            members.append(TrialSpec(t.nb_filters, t.kernel_size, t.pool_size, t.dense, t.lr, t.dropout,
                                     seed=len(members)))
    folds = [i % 5 for i in range(len(members))]
    x, yl = synthetic_mnist(60000, seed=0, device=dev)
    otr = torch.from_numpy(np.stack([kfold_split(60000, 5, f)[0] for f in folds])).to(dev)
    owner = lpt_assign([m.flops_per_sample_train() for m in members], 8)
    mine = [i for i, o in enumerate(owner) if o == 0]
    osub = otr[mine].contiguous()
    order = os.environ.get("ORDER", "full_first")
    if order == "sub_only":
        ballast = None
        if os.environ.get("BALLAST_GB"):   # untouched device memory held beside the share
            ballast = torch.empty(int(float(os.environ["BALLAST_GB"]) * 2**30), dtype=torch.uint8, device=dev)
            print(f"ballast {ballast.numel() / 2**30:.0f} GB", flush=True)
        sub = PopulationEngine([members[i] for i in mine], batch=100, device=dev)
        full = None
    elif order == "sub_first":
        sub = PopulationEngine([members[i] for i in mine], batch=100, device=dev)
        full = PopulationEngine(members, batch=100, device=dev)
    elif order == "full_then_free":
        full = PopulationEngine(members, batch=100, device=dev)
        sub = None
    else:
        full = PopulationEngine(members, batch=100, device=dev)
        sub = PopulationEngine([members[i] for i in mine], batch=100, device=dev)

    def timed(e, order, steps=10):
        for s_ in range(2):
            e.train_step(x, yl, order, s_ * e.batch)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for s_ in range(steps):
            e.train_step(x, yl, order, (s_ + 2) * e.batch)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / steps * 1e3

    print(f"engines created: {order}; device memory allocated {torch.cuda.memory_allocated(dev) / 2**30:.1f} GB",
          flush=True)
    if order == "full_then_free":   # time the whole population, free it, then time the share alone
        f0 = timed(full, otr)
        del full
        torch.cuda.synchronize(dev)
        if not os.environ.get("KEEP_CACHE"):   # KEEP_CACHE=1: the share reuses the freed engine's cached blocks
            torch.cuda.empty_cache()
        sub = PopulationEngine([members[i] for i in mine], batch=100, device=dev)
        for name in ("params", "grads", "act", "adam_m", "adam_v", "tables"):
            t = getattr(sub, name, None)
            if torch.is_tensor(t):
                print(f"  {name}: {t.numel() * t.element_size() / 2**20:.1f} MiB at 0x{t.data_ptr():x} "
                      f"(mod 2 MiB 0x{t.data_ptr() % (2 << 20):x})", flush=True)
        s0 = timed(sub, osub, 30)
        print(f"full, freed, then share: {s0:.2f} / {f0:.2f} ms = {s0 / f0:.4f}", flush=True)
        return
    if full is None:
        print(f"share alone: {timed(sub, osub, 30):.2f} ms", flush=True)
        return
    f1, s1 = timed(full, otr), timed(sub, osub)
    print(f"full then share: {s1:.2f} / {f1:.2f} ms = {s1 / f1:.4f}", flush=True)
    s2, f2 = timed(sub, osub), timed(full, otr)
    print(f"share then full: {s2:.2f} / {f2:.2f} ms = {s2 / f2:.4f}", flush=True)
    fs, ss = [], []
    for _ in range(5):
        fs.append(timed(full, otr, 4))
        ss.append(timed(sub, osub, 20))
    print(f"interleaved x5: {np.median(ss):.2f} / {np.median(fs):.2f} ms = {np.median(ss) / np.median(fs):.4f} "
          f"(share {' '.join(f'{v:.2f}' for v in ss)})", flush=True)


if __name__ == "__main__":
    main()
