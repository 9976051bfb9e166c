"""BASELINE configs[3] on 8 GPUs, projected from the MEASURED 1-GPU full search
(scripts/search_run.py ... --num-iterations 256 --epochs 10) -- a projection,
labelled as such, whose every term is a measured quantity of that run or of a
same-box probe:

* training: each population's measured 1-GPU training seconds x (ms per step of
  one GPU's LPT share of a 64-trial population, 40 members / ms per step of the
  whole 320-member population) -- the small-population efficiency measured by
  ``scripts/train_probe.py --shard 0/8`` and ``--trials 64`` on one box, not 1/8;
* chains: per population boundary, the 1-GPU chain work (its measured wait plus
  the part overlapped with training) spread over 8 GPUs, but never below the
  latency floor of the boundary's batches -- ceil(64 / (8 x workers)) rounds of
  the measured mean batch run time (``chain_run_s``);
* tells and the time between populations: as measured (they stay on rank 0).

    python scripts/project_configs3.py FULL.json --shard-ms 8.64 --full-ms 39.9 [--gpus 8]
"""
import argparse
import json
import math


def project(rep, shard_ms, full_ms, gpus=8):
    pops = rep["timeline"]              # [before, wait, train, trials] per population
    runs = rep.get("chain_run_s") or []
    workers = max(1, int(rep.get("chain_workers") or 1))
    factor = shard_ms / full_ms          # one GPU's share of a population vs the whole
    n_bound = max(1, len(pops) - 1)      # populations preceded by tells + ask batches
    tells_each = rep["tell_s"] / n_bound
    # chain_run_s[0] is the first ask (no told points: random initial points, no GP);
    # then one batch per launched trial of every later population
    out_pops, k, total = [], 1, 0.0
    for i, (before, wait, train, trials) in enumerate(pops):
        t_train = train * factor
        n_b = trials if i > 0 else 0     # one ask batch per launched trial after the first population
        batch_s = runs[k:k + n_b]
        k += n_b
        if batch_s:
            work = sum(batch_s) / workers            # 1-GPU seconds of chain work at `workers` concurrency
            floor = math.ceil(len(batch_s) / (gpus * workers)) * (sum(batch_s) / len(batch_s))
            t_chain = max(work / gpus, floor)
            t_tells = tells_each
        else:
            work = floor = t_chain = 0.0
            t_tells = before                         # the first population: startup asks as measured
        t = t_tells + t_chain + t_train
        out_pops.append({"trials": trials, "train_1gpu_s": train, "train_8gpu_s": t_train,
                         "chain_work_1gpu_s": work, "chain_floor_s": floor, "chain_8gpu_s": t_chain,
                         "rank0_tells_s": t_tells, "population_s": t})
        total += t
    told = rep["trials_told"]
    return {"workload": "BASELINE configs[3]: -n 129 --block-size 2 --n-fold 5 --num-iterations 256 --epochs 10 "
                        f"on {gpus} GPUs -- PROJECTION from the measured 1-GPU full run",
            "gpus": gpus, "train_factor": factor, "shard_ms_per_step": shard_ms, "full_ms_per_step": full_ms,
            "populations": out_pops, "wall_s": total, "told_trials": told,
            "told_trials_per_hour": told * 3600.0 / total,
            "trained_trials_per_hour": rep["trials_trained"] * 3600.0 / total,
            "optimizer_share": sum(p["chain_8gpu_s"] + p["rank0_tells_s"] for p in out_pops) / total,
            "measured_1gpu": {"wall_s": rep["wall_s"], "told_per_hour": rep["trials_per_hour"],
                              "optimizer_s": rep["optimizer_s"], "train_s": rep["train_s"]}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("report")
    ap.add_argument("--shard-ms", type=float, required=True)
    ap.add_argument("--full-ms", type=float, required=True)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rep = json.load(open(a.report))
    res = project(rep, a.shard_ms, a.full_ms, a.gpus)
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
