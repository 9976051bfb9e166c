#!/usr/bin/env python3
"""bench.py -- measures BASELINE.json's metric on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ei|train|all]

N=1 workload = BASELINE configs[1]: the GP/EI "ask" step, 200 observations,
10-dim space, 1M candidates, fp64.  One *step* = one full acquisition pass of the
hot path over the resident candidate batch: posterior + EI over every candidate
and the lowest-index top-k (skopt's argsort[:n_restarts]) -- for N>1 followed by
the RCCL all-gather of the per-rank (value, index) winners that yields the global
argmax (weak scaling: each rank scores its own 1M candidates).

Prints ONE JSON line on rank 0.  Multi-GPU: launched by torch.distributed.run,
one rank per GPU, barrier + synchronize around the timed region, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 (vector = matrix rate on gfx950), AMD spec
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 MFMA / vector, MI355X_MICROARCH.md:42
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md:36 (spec)


def ei_flops_per_candidate(n, d):
    """Algorithmic FLOPs of the device formulation per candidate:
    distances N*3D, Matern N*8, mu 2N, triangular V = K* L^-T  N(N+1), ||V||^2 2N,
    acquisitions ~30."""
    return n * (n + 1) + n * (3 * d + 12) + 30


def ei_bytes_per_candidate(d, k_vals=1):
    """Algorithmic HBM bytes: candidate row in, mu + sd + one acquisition row out."""
    return 8 * d + 8 * (2 + k_vals)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def load_traffic(kernel, config_key):
    """HBM bytes per launch from the committed PMC summary (profiles/), if present
    for exactly this kernel + workload; else None."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        d = json.load(open(path))
        e = d.get(kernel, {}).get(config_key)
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


def cpu_baseline_ei(n=200, d=10, sample=150_000):
    """skopt's literal K_inv einsum posterior + EI (the oracle restatement) timed on
    the host: single-threaded einsum, as skopt calls it."""
    from oracle import gp_ei as O

    X, y = O.synthetic_problem(n, d, 0)
    st = O.gp_from_theta(X, y, 17.4955, np.array([16.2, 1.91, 1.65, 9.84, 1.84, 2.94, 2.45, 9.09, 8.13, 1.94]),
                         0.0465)
    C = O.synthetic_candidates(sample, d, seed=11)
    t0 = time.perf_counter()
    mu, sd = O.posterior_skopt(st, C)
    v = -O.gaussian_ei(mu, sd, float(np.min(y)))
    np.argsort(v)[:5]
    dt = time.perf_counter() - t0
    return {"value": sample / dt, "unit": "candidates/s", "cores": 1, "kind": "port",
            "sample": f"{sample} candidates, N={n} D={d}, skopt K_inv einsum form (oracle/gp_ei.py), "
                      f"{dt:.1f} s on 1 host core"}


def bench_ei(args, torch, dist, ws, rank, dev):
    from oracle import gp_ei as O  # noqa: F401  (only for the fixed synthetic recipe)
    from mpi_opt_amd.gp import DeviceGP

    n, d, m, k = 200, 10, args.candidates, 5
    X, y = O.synthetic_problem(n, d, 0)
    # hyper-parameters as fitted by sklearn on this data (tests/golden/gp_ei_n200_d10.npz)
    ls = np.array([16.2, 1.91, 1.65, 9.84, 1.84, 2.94, 2.45, 9.09, 8.13, 1.94])
    g = DeviceGP(X, y, 17.4955, ls, 0.0465, device=dev)
    cand = torch.from_numpy(O.synthetic_candidates(m, d, seed=1 + rank)).to(dev)
    y_opt = float(np.min(y))
    torch.cuda.synchronize(dev)

    gathered = torch.empty(ws, 2, dtype=torch.float64, device=dev) if ws > 1 else None

    def step():
        out = g.score(cand, y_opt, acqs=("EI",), k=k, want_mu_sd=True, want_values=True)
        if ws > 1:
            idx, val = out["topk"]["EI"]
            local = torch.stack([val[0], (idx[0] + rank * m).to(torch.float64)])
            dist.all_gather_into_tensor(gathered, local)
        return out

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # dominant kernel alone (k=0: no top-k merge), HIP events on its stream
    stream = torch.cuda.current_stream(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    reps = max(args.steps, 5)
    e0.record(stream)
    for _ in range(reps):
        g.score(cand, y_opt, acqs=("EI",), k=0, want_mu_sd=True, want_values=True)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    t_kernel = e0.elapsed_time(e1) / 1e3 / reps

    flops = ei_flops_per_candidate(n, d) * m
    algo_bytes = ei_bytes_per_candidate(d) * m
    achieved = flops / t_kernel / 1e12
    value = ws * m * args.steps / dt
    res = {
        "metric": "EI candidates/sec (GP/EI ask step, N=200 obs, D=10, fp64)",
        "value": value,
        "unit": "candidates/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY §8d recipe: X~U[0,1]^{200x10}, y=sin(Xw)+0.1eps; candidates~U[0,1]^{1Mx10})",
        "config": {"workload": "BASELINE configs[1]: GP/EI ask step, 200 observations, 10-dim, "
                               f"{m} candidates per GPU, top-{k} (skopt argsort[:n_restarts])",
                   "n_obs": n, "dims": d, "candidates_per_gpu": m,
                   "parallelism": f"candidates sharded, {ws} GPU(s), all-gather of (value,index)"},
        "roofline": {"kernel": "gp_score_kernel", "bound": "mfma", "achieved": achieved,
                     "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                     "traffic": load_traffic("gp_score_kernel", f"n{n}_d{d}_m{m}"),
                     "kernel_ms": t_kernel * 1e3,
                     "algorithmic_flops_per_launch": flops,
                     "algorithmic_hbm_bytes_per_launch": algo_bytes,
                     "algorithmic_hbm_gbs": algo_bytes / t_kernel / 1e9},
    }
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="ei", choices=["ei"])
    ap.add_argument("--candidates", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch

    ws, rank, local = dist_env()
    dist = None
    if ws > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local if ws > 1 else 0)
    if ws == 1 and args.gpus != 1:
        print(f"warning: --gpus {args.gpus} without torch.distributed.run; running 1 GPU", file=sys.stderr)

    res = bench_ei(args, torch, dist, ws, rank, dev)
    if rank == 0:
        if ws == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline_ei()
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
