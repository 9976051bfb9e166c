"""A/B the population plan knobs (env, read at plan creation) on the 320-member
training workload in one process; prints per-phase device ms per train step."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd.population import PopulationEngine, TrialSpec, kfold_split, synthetic_mnist  # noqa: E402
from scripts.train_probe import sample_trials  # noqa: E402

ARGS = sys.argv[1:]
SHARD = None
if ARGS and ARGS[0].startswith("--shard="):     # --shard=K/N: one GPU's LPT share of the population
    SHARD = tuple(int(v) for v in ARGS.pop(0).split("=", 1)[1].split("/"))
VARIANTS = [v for v in (ARGS or ["base"])]


def members_of(trials, folds=5):
    out = []
    for t in trials:
        for f in range(folds):
            out.append(TrialSpec(t.nb_filters, t.kernel_size, t.pool_size, t.dense, t.lr, t.dropout, seed=len(out)))
    return out


def run(variant, x, y, order, members, steps=3):
    # a variant is "base" or MPO_POP_PLAN's "key=value,..." (planner overrides, csrc/cnn.hip plan_knob)
    env = {} if variant == "base" else {"MPO_POP_PLAN": variant}
    env.setdefault("MPO_POP_PROFILE", "1")
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        eng = PopulationEngine(members, batch=100)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    eng.train_step(x, y, order, 0)
    torch.cuda.synchronize()
    eng.profile(reset=True)
    t0 = time.time()
    for s in range(steps):
        eng.train_step(x, y, order, (s + 1) * 100)
    torch.cuda.synchronize()
    wall = (time.time() - t0) / steps * 1e3
    prof = {k: v / steps for k, v in eng.profile(reset=True).items()}
    loss = float(eng.loss[:8].mean())
    del eng
    torch.cuda.empty_cache()
    return wall, prof, loss


def main():
    members = members_of(sample_trials(64))
    if SHARD:
        from mpi_opt_amd.blocks import lpt_assign

        owner = lpt_assign([m.flops_per_sample_train() for m in members], SHARD[1])
        members = [m for m, o in zip(members, owner) if o == SHARD[0]]
    x, y = synthetic_mnist(60000, seed=0)
    tr = np.stack([kfold_split(60000, 5, i % 5)[0] for i in range(len(members))])
    order = torch.from_numpy(tr).cuda()
    flops = sum(m.flops_per_sample_train() for m in members) * 100
    for v in VARIANTS:
        wall, prof, loss = run(v, x, y, order, members)
        tot = sum(prof.values())
        print(f"== {v}: {wall:.2f} ms/step wall, {tot:.2f} ms device, {flops / (tot / 1e3) / 157.3e12 * 100:.1f}% FP32 peak, loss {loss:.5f}")
        groups = {}
        for k, ms in prof.items():
            groups.setdefault(k.split("/")[0], 0.0)
            groups[k.split("/")[0]] += ms
        print("   " + "  ".join(f"{k}={ms:.2f}" for k, ms in sorted(groups.items(), key=lambda kv: -kv[1])))
        print("   " + "  ".join(f"{k}={ms:.2f}" for k, ms in prof.items() if "/" in k and ms > 0.05), flush=True)


if __name__ == "__main__":
    main()
