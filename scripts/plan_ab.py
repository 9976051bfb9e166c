"""Same-process A/B of population-plan variants (MPO_POP_PLAN strings).

One engine per variant over the same members and the same init, timed in
interleaved rounds (guide §5.4 rule 24), and the per-member losses of every
variant compared bit for bit against the first one after the same steps
(plan knobs only re-cut or re-order work, so they must not move a bit).

  python scripts/plan_ab.py --variants "xcd=0" "xcd=1" --rounds 5 --steps 5
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401
from mpi_opt_amd.population import PopulationEngine, TrialSpec, kfold_split, synthetic_mnist  # noqa: E402
from scripts.train_probe import sample_trials  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", required=True)
    ap.add_argument("--trials", type=int, default=64)
    ap.add_argument("--folds", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--shard", default=None, help="K/N: rank K's LPT share over N ranks")
    args = ap.parse_args()
    members, folds = [], []
    for t in sample_trials(args.trials):
        for f in range(args.folds):
            members.append(TrialSpec(t.nb_filters, t.kernel_size, t.pool_size, t.dense, t.lr, t.dropout,
                                     seed=len(members)))
            folds.append(f)
    if args.shard:
        from mpi_opt_amd.blocks import lpt_assign

        k, n = (int(v) for v in args.shard.split("/"))
        owner = lpt_assign([m.flops_per_sample_train() for m in members], n)
        mine = [i for i, o in enumerate(owner) if o == k]
        members, folds = [members[i] for i in mine], [folds[i] for i in mine]
    x, y = synthetic_mnist(60000, seed=0)
    order = torch.from_numpy(np.stack([kfold_split(60000, args.folds, f)[0] for f in folds])).cuda()
    engines = []
    for v in args.variants:
        os.environ["MPO_POP_PLAN"] = v
        engines.append(PopulationEngine(members, batch=100))
    os.environ.pop("MPO_POP_PLAN", None)
    flops = sum(m.flops_per_sample_train() for m in members) * 100
    times = [[] for _ in engines]
    pos = [0] * len(engines)
    for e in engines:   # warm-up
        for _ in range(2):
            e.train_step(x, y, order, pos[0] * 100)
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for i, e in enumerate(engines):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for s in range(args.steps):
                e.train_step(x, y, order, ((r * args.steps + s) % 400) * 100)
            torch.cuda.synchronize()
            times[i].append((time.perf_counter() - t0) / args.steps * 1e3)
    ref = engines[0].loss.cpu().numpy()
    print(f"members={len(members)} rounds={args.rounds} steps/round={args.steps}")
    for i, v in enumerate(args.variants):
        t = np.array(times[i])
        same = bool(np.array_equal(engines[i].loss.cpu().numpy(), ref))
        print(f"{v:40s} median {np.median(t):8.3f} ms  min {t.min():8.3f}  "
              f"frac {flops / (np.median(t) / 1e3) / 157.3e12:.4f}  loss bits == variant 0: {same}", flush=True)


if __name__ == "__main__":
    main()
