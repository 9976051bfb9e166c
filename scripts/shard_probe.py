"""A GPU's share of a population (the 8-GPU search's training term): step time
with the plan's streams, then the per-phase split (MPO_POP_PROFILE=2, serial).
``--labels-ab`` instead times a long run of the whole population on uniform vs
learnable synthetic labels in windows (data-dependent clocks)."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd.blocks import lpt_assign  # noqa: E402
from mpi_opt_amd.population import PopulationEngine, TrialSpec, kfold_split, synthetic_mnist  # noqa: E402
from scripts.train_probe import sample_trials  # noqa: E402


def members_of(trials, folds, shard, bench_set=False):
    members, fl = [], []
    if bench_set:   # bench.py's own draw (lr and dropout drawn between the shapes): its train leg's population
        from bench import sample_trials as bench_sample_trials
        drawn = bench_sample_trials(trials, seed=13579)
    else:
        drawn = sample_trials(trials)
    for t in drawn:
        for f in range(folds):
            members.append(TrialSpec(t.nb_filters, t.kernel_size, t.pool_size, t.dense, t.lr, t.dropout,
                                     seed=len(members)))
            fl.append(f)
    if shard:
        k, n = (int(v) for v in shard.split("/"))
        owner = lpt_assign([m.flops_per_sample_train() for m in members], n)
        mine = [i for i, o in enumerate(owner) if o == k]
        members, fl = [members[i] for i in mine], [fl[i] for i in mine]
    return members, fl


def timed(eng, x, y, order, steps, s0=2):
    for s in range(2):
        eng.train_step(x, y, order, s * 100)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        eng.train_step(x, y, order, ((s + s0) % 400) * 100)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=64)
    ap.add_argument("--folds", type=int, default=5)
    ap.add_argument("--shard", default="0/8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--labels-ab", action="store_true")
    ap.add_argument("--bench-set", action="store_true", help="bench.py's train-leg trials instead of train_probe's")
    args = ap.parse_args()
    if args.labels_ab:
        members, fl = members_of(args.trials, args.folds, None)
        for labels in ("uniform", "learnable", "uniform"):
            x, y = synthetic_mnist(60000, seed=0, labels=labels)
            order = torch.from_numpy(np.stack([kfold_split(60000, args.folds, f)[0] for f in fl])).cuda()
            eng = PopulationEngine(members, batch=100)
            win = []
            for w in range(6):
                win.append(timed(eng, x, y, order, args.steps, s0=2 + w * args.steps) * 1e3)
            print(f"labels {labels:9s} ms/step by window of {args.steps}: " + " ".join(f"{v:.2f}" for v in win),
                  "loss", float(eng.loss.mean()), flush=True)
            del eng
        return
    members, fl = members_of(args.trials, args.folds, args.shard, args.bench_set)
    x, y = synthetic_mnist(60000, seed=0)
    order = torch.from_numpy(np.stack([kfold_split(60000, args.folds, f)[0] for f in fl])).cuda()
    eng = PopulationEngine(members, batch=100)
    dt = timed(eng, x, y, order, args.steps)
    nts = np.bincount([(m.nb_filters + 15) // 16 for m in members], minlength=5)[1:]
    print(f"shard {args.shard}: {len(members)} members, NT histogram {nts.tolist()}, {dt * 1e3:.2f} ms/step (streams)",
          flush=True)
    del eng
    os.environ["MPO_POP_PROFILE"] = "2"
    eng = PopulationEngine(members, batch=100)
    dts = timed(eng, x, y, order, args.steps)
    prof = eng.profile()
    print(f"serial (profiled) {dts * 1e3:.2f} ms/step; per phase, ms per step:")
    for name, ms in sorted(prof.items(), key=lambda kv: -kv[1]):
        print(f"  {name:40s} {ms / (args.steps + 2):8.3f}")


if __name__ == "__main__":
    main()
