"""Same-process A/B of DenseNet population plan variants (MPO_DN_PLAN strings):
one population per variant over the same members, init and data, timed in
interleaved rounds; parameters after the same steps compared bit for bit.

  python scripts/dn_ab.py --variants "wg1v=0" "wg1v=1" --rounds 5 --steps 5
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_opt_amd.densenet import DenseNetArch, DenseNetPopulation, flops_per_sample_train, synthetic_cifar  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--members", type=int, default=32)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    x, y = synthetic_cifar(n=5000, seed=0)
    g = torch.Generator(device="cuda").manual_seed(0)
    order = torch.stack([torch.randperm(5000, device="cuda", dtype=torch.int64, generator=g).to(torch.int32)
                         for _ in range(args.members)])
    lrs = list(10.0 ** np.random.RandomState(0).uniform(-5, -1, args.members))
    pops = []
    for v in args.variants:
        os.environ["MPO_DN_PLAN"] = v
        pops.append(DenseNetPopulation(DenseNetArch(), lrs, batch=args.batch))
    os.environ.pop("MPO_DN_PLAN", None)
    fl = flops_per_sample_train(pops[0].layers) * args.batch * args.members
    for p in pops:
        for s in range(2):
            p.train_step(x, y, order, s * args.batch)
    torch.cuda.synchronize()
    times = [[] for _ in pops]
    for r in range(args.rounds):
        for i, p in enumerate(pops):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for s in range(args.steps):
                p.train_step(x, y, order, ((2 + r * args.steps + s) % 40) * args.batch)
            torch.cuda.synchronize()
            times[i].append((time.perf_counter() - t0) / args.steps * 1e3)
    ref = pops[0].params.cpu().numpy()
    for i, v in enumerate(args.variants):
        t = np.array(times[i])
        same = bool(np.array_equal(pops[i].params.cpu().numpy(), ref))
        print(f"{v:30s} train step median {np.median(t):7.3f} ms  min {t.min():7.3f}  "
              f"frac {fl / (np.median(t) / 1e3) / 157.3e12:.4f}  params bits == variant 0: {same}", flush=True)


if __name__ == "__main__":
    main()
