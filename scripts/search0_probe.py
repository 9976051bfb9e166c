"""configs[0] populations (the reference's own mnist search: -n 21 --block-size 5,
10 random trials trained as populations [4, 4, 2] x 5 folds) timed per train step
under plan-knob variants, all in one process (same box, same data).

    python scripts/search0_probe.py base dg_tiles=16 conv_mt=2
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd.models import mnist_space  # noqa: E402
from mpi_opt_amd.optimizer import Optimizer  # noqa: E402
from mpi_opt_amd.population import PopulationEngine, TrialSpec, kfold_split, synthetic_mnist  # noqa: E402


def search0_populations():
    """The 10 initial (random) points of the configs[0] search, grouped as the
    scheduler launches them (pop(-1) order, 4 blocks)."""
    X = Optimizer(mnist_space(), base_estimator="dummy", random_state=13579).ask(10)
    X = X[::-1]
    return [X[0:4], X[4:8], X[8:10]]


def members_of(params):
    out = []
    for p in params:
        nb, ps, ks, dense, dr = p
        for f in range(5):
            out.append(TrialSpec(int(nb), int(ks), int(ps), int(dense), 1e-3, float(dr), seed=len(out)))
    return out


def run(variant, pops, x, y, steps=60, evals=10, profile=False):
    # a variant is "base" or MPO_POP_PLAN's "key=value,..." (planner overrides, csrc/cnn.hip plan_knob)
    env = {} if variant == "base" else {"MPO_POP_PLAN": variant}
    if profile:
        env["MPO_POP_PROFILE"] = "1"   # per-launch HIP events (adds a little host time per step)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    res = []
    try:
        for params in pops:
            members = members_of(params)
            eng = PopulationEngine(members, batch=100)
            tr = np.stack([kfold_split(60000, 5, i % 5)[0] for i in range(len(members))])
            va = np.stack([kfold_split(60000, 5, i % 5)[1] for i in range(len(members))])
            order, vorder = torch.from_numpy(tr).cuda(), torch.from_numpy(va).cuda()
            for s in range(3):
                eng.train_step(x, y, order, s * 100)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for s in range(steps):
                eng.train_step(x, y, order, (s + 3) * 100)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for s in range(evals):
                eng.eval_step(x, y, vorder, s * 100)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res.append(((t1 - t0) / steps * 1e3, (t2 - t1) / evals * 1e3, float(eng.loss.mean())))
            if profile:
                prof = eng.profile(reset=True)
                groups = {}
                for k, ms in prof.items():
                    groups[k.split("/")[0]] = groups.get(k.split("/")[0], 0.0) + ms / (steps + evals + 3)
                print(f"   {variant} population of {len(members)} members, device ms per step: "
                      + "  ".join(f"{k}={v:.3f}" for k, v in sorted(groups.items(), key=lambda kv: -kv[1])),
                      flush=True)
            del eng
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return res


def main():
    pops = search0_populations()
    x, y = synthetic_mnist(60000, seed=0)
    for p in pops:
        print("population", [[round(float(v), 3) for v in q] for q in p], flush=True)
    variants = sys.argv[1:] or ["base"]
    for v in variants:
        run(v, pops, x, y, steps=20, evals=5, profile=True)
    for rep in range(2):
        for v in variants:
            res = run(v, pops, x, y)
            # a fold-epoch is 480 train steps + 120 validation batches; the search trains 10 epochs
            est = sum(10 * (480 * tr + 120 * ev) for tr, ev, _ in res) / 1e3
            print(f"[{rep}] {v:>28}: " + "  ".join(f"pop{i}: {tr:.3f} ms/step eval {ev:.3f} (loss {ls:.4f})"
                                                  for i, (tr, ev, ls) in enumerate(res))
                  + f"  -> search training {est:.1f} s", flush=True)


if __name__ == "__main__":
    main()
