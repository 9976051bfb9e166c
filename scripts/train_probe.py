"""Time the population train step on one GPU (diagnostic; bench.py has the contract)."""
import argparse
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd.population import PopulationEngine, TrialSpec, kfold_split, synthetic_mnist  # noqa: E402


def sample_trials(n, seed=13579):
    rng = np.random.RandomState(seed)
    out = []
    for i in range(n):
        out.append(TrialSpec(nb_filters=int(rng.randint(10, 51)), pool_size=int(rng.randint(2, 11)),
                             kernel_size=int(rng.randint(2, 11)), dense=int(rng.randint(50, 201)), seed=i))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=64)
    ap.add_argument("--folds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--shard", default=None,
                    help="K/N: only rank K's LPT-by-FLOPs share of the (trial, fold) units over N ranks "
                         "(what one GPU trains of the population in the distributed search)")
    ap.add_argument("--no-eval", action="store_true",
                    help="train steps only (bench.py's PMC passes divide by the train steps)")
    args = ap.parse_args()
    trials = sample_trials(args.trials)
    members = []
    folds = []
    for t in trials:
        for f in range(args.folds):
            members.append(TrialSpec(t.nb_filters, t.kernel_size, t.pool_size, t.dense, t.lr, t.dropout, seed=len(members)))
            folds.append(f)
    if args.shard:
        from mpi_opt_amd.blocks import lpt_assign

        k, n = (int(v) for v in args.shard.split("/"))
        owner = lpt_assign([m.flops_per_sample_train() for m in members], n)
        mine = [i for i, o in enumerate(owner) if o == k]
        members = [members[i] for i in mine]
        folds = [folds[i] for i in mine]
    t0 = time.time()
    eng = PopulationEngine(members, batch=100)
    x, y = synthetic_mnist(60000, seed=0)
    tr = np.stack([kfold_split(60000, args.folds, f)[0] for f in folds])
    order = torch.from_numpy(tr).cuda()
    torch.cuda.synchronize()
    print("setup %.1fs members=%d params=%.1fM act=%.2fGB" % (time.time() - t0, len(members), eng.n_params / 1e6,
                                                              eng.act.numel() * 4 / 1e9), flush=True)
    for s in range(2):
        eng.train_step(x, y, order, s * 100)
    torch.cuda.synchronize()
    t0 = time.time()
    for s in range(args.steps):
        eng.train_step(x, y, order, (s + 2) * 100)
    torch.cuda.synchronize()
    dt = (time.time() - t0) / args.steps
    flops = sum(m.flops_per_sample_train() for m in members) * 100
    print("train step %.2f ms  %.1f TFLOP/s  (%.1f%% of 157.3)" % (dt * 1e3, flops / dt / 1e12, flops / dt / 157.3e12 * 100))
    print("loss", eng.loss[:5].cpu().numpy())
    if __import__("os").environ.get("MPO_POP_PROFILE"):
        ph = eng.profile()   # ms summed over the 12 steps (serial: profiled steps stay on one stream)
        tot = sum(ph.values())
        for k_, v_ in sorted(ph.items(), key=lambda kv: -kv[1]):
            print(f"  {k_:28s} {v_ / 12:8.3f} ms/step  {100 * v_ / tot:5.1f}%")
    if args.no_eval:
        return
    va = np.stack([kfold_split(60000, args.folds, f)[1] for f in folds])
    vorder = torch.from_numpy(va).cuda()
    eng.eval_step(x, y, vorder, 0)
    torch.cuda.synchronize()
    t0 = time.time()
    for s in range(args.steps):
        eng.eval_step(x, y, vorder, (s + 1) * 100)
    torch.cuda.synchronize()
    de = (time.time() - t0) / args.steps
    fe = sum(m.flops_per_sample_fwd() for m in members) * 100
    print("eval step %.2f ms  %.1f TFLOP/s  (%.1f%% of 157.3)" % (de * 1e3, fe / de / 1e12, fe / de / 157.3e12 * 100))


if __name__ == "__main__":
    main()
