#!/usr/bin/env python3
"""bench.py -- measures BASELINE.json's metric on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload ei|train|densenet|all]

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
import collections
import gc
import math
import json
import os
import random
import shutil
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


PMC_FAMILIES = (("conv_img_kernel<0", "conv1_fwd"), ("conv_img_kernel<1", "conv2_fwd"), ("conv_dgrad", "conv2_dgrad"),
                ("conv_wgrad_kernel<1", "conv2_wgrad"), ("conv_wgrad_kernel<0", "conv1_wgrad"),
                ("dense_kernel", "dense_kernel"))
# DenseNet kernels that issue MFMAs (csrc/densenet.hip): the convs (3x3 growth / initial,
# 1x1 transitions, their input gradients) and the two weight-gradient kernels
DN_PMC_FAMILIES = (("dn_conv_kernel<3", "conv3x3"), ("dn_conv_kernel<1", "conv1x1"), ("dn_conv1x1_kernel", "conv1x1"),
                   ("dn_wgrad3_kernel", "wgrad3"), ("dn_wgrad1_kernel", "wgrad1"))


def mfma_busy(rows, families):
    """SQ_VALU_MFMA_BUSY_CYCLES over the SIMD cycles of the matching dispatches
    (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), per family and pooled."""
    acc, num, den = {}, 0.0, 0.0
    for needle, fam in families:
        busy = sum(_per_dispatch(rows, "SQ_VALU_MFMA_BUSY_CYCLES", lambda k: needle in k).values())
        gui = sum(_per_dispatch(rows, "GRBM_GUI_ACTIVE", lambda k: needle in k).values())
        if gui:
            b0, g0 = acc.get(fam, (0.0, 0.0))
            acc[fam] = (b0 + busy, g0 + gui / 8 * 1024)   # families sharing a label are pooled
            num += busy
            den += gui / 8 * 1024
    return (num / den if den else None), {f: b / g for f, (b, g) in acc.items()}


def pmc_pass(counters, prog, timeout=150):
    """One ``rocprofv3 --pmc`` pass (its own process, counters of one pass only)
    over ``python <prog>``; returns the counter_collection rows, or raises."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    d = tempfile.mkdtemp(prefix="mpo_pmc_", dir="/tmp")
    try:
        cmd = ["rocprofv3", "--pmc", *counters, "-d", d, "-o", "pmc", "--output-format", "csv", "--",
               sys.executable, *prog]
        r = subprocess.run(cmd, cwd="/tmp", env={**os.environ, "TMPDIR": "/tmp"}, stdout=subprocess.DEVNULL,
                           stderr=subprocess.PIPE, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError(f"rocprofv3 exit {r.returncode}: {r.stderr.decode(errors='replace')[-300:]}")
        paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not paths:
            raise RuntimeError("rocprofv3 wrote no counter_collection.csv")
        return list(csv.DictReader(open(paths[0])))
    finally:
        shutil.rmtree(d, ignore_errors=True)


def kernel_trace_pass(prog, match, timeout=150):
    """One ``rocprofv3 --kernel-trace --stats`` run (its own process) over ``python
    <prog>``: (calls, average ns) of the kernels whose name matches, from the
    kernel_stats summary -- the same figure the committed profiles/ summaries hold."""
    import csv
    import glob
    import subprocess
    import tempfile

    d = tempfile.mkdtemp(prefix="mpo_kt_", dir="/tmp")
    try:
        cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "kt", "--output-format", "csv", "--",
               sys.executable, *prog]
        r = subprocess.run(cmd, cwd="/tmp", env={**os.environ, "TMPDIR": "/tmp"}, stdout=subprocess.DEVNULL,
                           stderr=subprocess.PIPE, timeout=timeout)
        if r.returncode != 0:
            raise RuntimeError(f"rocprofv3 exit {r.returncode}: {r.stderr.decode(errors='replace')[-300:]}")
        paths = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if not paths:
            raise RuntimeError("rocprofv3 wrote no kernel_stats.csv")
        calls, total = 0, 0.0
        for row in csv.DictReader(open(paths[0])):
            if match(row["Name"]):
                calls += int(row["Calls"])
                total += float(row["TotalDurationNs"])
        return calls, (total / calls if calls else None)
    finally:
        shutil.rmtree(d, ignore_errors=True)


def _per_dispatch(rows, counter, match):
    vals = collections.defaultdict(float)
    for r in rows:
        if r["Counter_Name"] == counter and match(r["Kernel_Name"]):
            vals[r.get("Dispatch_Id", r.get("Correlation_Id"))] += float(r["Counter_Value"])
    return vals


def _kernel_family(name):
    """'void (anonymous namespace)::conv_dgrad_kernel<3>(...)' -> 'conv_dgrad_kernel<3>'."""
    n = name.split("::", 1)[1] if "::" in name else name
    return n.split("(", 1)[0]


def _per_kernel_bytes(rows_f, rows_w, match, steps, top=12, family=False):
    """HBM bytes per step by kernel instance (FETCH_SIZE x 2 + WRITE_SIZE), largest
    first; ``family`` sums the template instances of a kernel (all of them, no top cut)."""
    by = collections.defaultdict(float)
    for rows, counter, mult in ((rows_f, "FETCH_SIZE", 2.0), (rows_w, "WRITE_SIZE", 1.0)):
        for r in rows:
            if r["Counter_Name"] == counter and match(r["Kernel_Name"]):
                name = _kernel_family(r["Kernel_Name"])
                by[name.split("<", 1)[0] if family else name] += mult * 1024.0 * float(r["Counter_Value"]) / steps
    items = sorted(by.items(), key=lambda kv: -kv[1])
    return dict(items if family else items[:top])


def live_pmc(train_trials):
    """HBM traffic measured in this run (MI355X_MICROARCH.md HBM section): separate
    FETCH_SIZE and WRITE_SIZE passes (KiB; FETCH_SIZE doubled -- gfx950 reports half
    of a wide streaming read), per launch of gp_score_kernel over scripts/ei_probe.py
    (the bench's EI step, 3 launches) and per train step over scripts/train_probe.py
    (the bench's 320-member population, 3 train steps), plus one SQ pass for the
    training kernels' MFMA-busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over
    GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs).  Runs before this process touches the
    GPU.  Returns {"ei": ..., "train": ...}; a failed pass leaves its entry None
    with the reason."""
    out = {"ei": None, "train": None, "densenet": None, "errors": []}
    ei_prog = [os.path.join(ROOT, "scripts", "ei_probe.py"), "3"]
    try:
        # one acquisition pass = gp_score_kernel (r03: the posterior / acquisition /
        # top-k finish runs inside it over the workgroup's own (mu_n, q) rows, the only
        # non-algorithmic traffic; score_finish_kernel of earlier rounds kept matching)
        acq = lambda k: "gp_score_kernel" in k or "score_finish_kernel" in k   # noqa: E731
        f = _per_dispatch(pmc_pass(["FETCH_SIZE"], ei_prog), "FETCH_SIZE", acq)
        w = _per_dispatch(pmc_pass(["WRITE_SIZE"], ei_prog), "WRITE_SIZE", acq)
        passes = 3
        fetch = 1024.0 * sum(f.values()) / passes
        write = 1024.0 * sum(w.values()) / passes
        out["ei"] = {"hbm_bytes_per_launch": 2.0 * fetch + write, "fetch_size_bytes_raw": fetch,
                     "write_size_bytes": write, "launches": passes, "dispatches": len(f)}
        # the dominant kernel's average duration as rocprofv3 reports it (kernel-trace
        # stats) over the bench's own EI leg in a child process (the same sustained
        # launches: a short probe runs at a higher clock -- 0.96 vs 1.31 ms measured);
        # the roofline's HIP-event time is measured in this process beside it
        calls, avg_ns = kernel_trace_pass([os.path.join(ROOT, "bench.py"), "--workload", "ei", "--no-pmc",
                                           "--no-cpu-baseline"], lambda k: "gp_score_kernel" in k, timeout=300)
        out["ei"]["rocprof_calls"], out["ei"]["rocprof_avg_ns"] = calls, avg_ns
    except Exception as e:  # noqa: BLE001 -- reported, the bench line carries traffic null
        out["errors"].append(f"ei: {e}")
    # 2 warmup + 1 timed train steps and no evaluation (r04 counted the probe's eval
    # kernels too, which inflated the forward families 5/3x)
    steps = 3
    tr_prog = [os.path.join(ROOT, "scripts", "train_probe.py"), "--steps", "1", "--trials", str(train_trials),
               "--no-eval"]
    try:
        ours = lambda k: "anonymous namespace" in k     # noqa: E731 -- libmpo's kernels, not torch's setup
        rf, rw = pmc_pass(["FETCH_SIZE"], tr_prog), pmc_pass(["WRITE_SIZE"], tr_prog)
        f = _per_dispatch(rf, "FETCH_SIZE", ours)
        w = _per_dispatch(rw, "WRITE_SIZE", ours)
        per_kernel = _per_kernel_bytes(rf, rw, ours, steps)
        per_family = _per_kernel_bytes(rf, rw, ours, steps, family=True)
        fetch = 1024.0 * sum(f.values()) / steps
        write = 1024.0 * sum(w.values()) / steps
        busy, per = mfma_busy(pmc_pass(["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"], tr_prog), PMC_FAMILIES)
        out["train"] = {"hbm_bytes_per_train_batch": 2.0 * fetch + write, "fetch_size_bytes_raw": fetch,
                        "write_size_bytes": write, "mfma_busy": busy, "steps_counted": steps,
                        "per_kernel_mfma_busy": per, "per_kernel_hbm_bytes": per_kernel,
                        "per_family_hbm_bytes": per_family}
    except Exception as e:  # noqa: BLE001
        out["errors"].append(f"train: {e}")
    # DenseNet (configs[4]): 2 warmup + 3 train steps of the 32-member population
    dn_prog = [os.path.join(ROOT, "scripts", "dn_probe.py"), "--steps", "3", "--no-eval"]
    try:
        ours = lambda k: "anonymous namespace" in k     # noqa: E731
        rf, rw = pmc_pass(["FETCH_SIZE"], dn_prog), pmc_pass(["WRITE_SIZE"], dn_prog)
        f = _per_dispatch(rf, "FETCH_SIZE", ours)
        w = _per_dispatch(rw, "WRITE_SIZE", ours)
        fetch = 1024.0 * sum(f.values()) / 5
        write = 1024.0 * sum(w.values()) / 5
        busy, per = mfma_busy(pmc_pass(["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"], dn_prog), DN_PMC_FAMILIES)
        out["densenet"] = {"hbm_bytes_per_train_step": 2.0 * fetch + write, "fetch_size_bytes_raw": fetch,
                           "write_size_bytes": write, "steps": 5, "mfma_busy": busy, "per_kernel_mfma_busy": per,
                           "per_kernel_hbm_bytes": _per_kernel_bytes(rf, rw, ours, 5),
                           "per_family_hbm_bytes": _per_kernel_bytes(rf, rw, ours, 5, family=True)}
    except Exception as e:  # noqa: BLE001
        out["errors"].append(f"densenet: {e}")
    return out


def host_cores():
    """Host cores this job may use: the box's share (OMP_NUM_THREADS is set to it
    there), else the affinity mask."""
    return int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))


def cpu_baseline_ei(n=200, d=10, sample_1core=100_000):
    """skopt's literal K_inv einsum posterior + EI + argsort (the oracle
    restatement; skopt calls it single-threaded) timed on the host: on one core,
    and split over every host core (one single-threaded process per core).
    ``value`` is the all-cores rate."""
    from oracle import gp_ei as O

    X, y = O.synthetic_problem(n, d, 0)
    amp, ls, noise = 17.4955, np.array([16.2, 1.91, 1.65, 9.84, 1.84, 2.94, 2.45, 9.09, 8.13, 1.94]), 0.0465
    st = O.gp_from_theta(X, y, amp, ls, noise)
    C = O.synthetic_candidates(sample_1core, d, seed=11)
    t0 = time.perf_counter()
    mu, sd = O.posterior_skopt(st, C)
    v = -O.gaussian_ei(mu, sd, float(np.min(y)))
    np.argsort(v)[:5]
    dt1 = time.perf_counter() - t0
    cores = host_cores()
    sample_all = int(sample_1core * min(cores, 16) // 2)
    dt, done = O.time_skopt_ei(X, y, amp, ls, noise, sample_all, cores)
    return {"value": done / dt, "unit": "candidates/s", "cores": cores, "kind": "port",
            "single_core": sample_1core / dt1,
            "sample": f"{done} candidates over {cores} single-threaded processes ({dt:.1f} s) and "
                      f"{sample_1core} on 1 core ({dt1:.1f} s, {sample_1core / dt1:.3g} cand/s); N={n} D={d}, "
                      f"skopt K_inv einsum form + EI + argsort (oracle/gp_ei.py)"}


def bench_ei(args, torch, dist, ws, rank, dev):
    from mpi_opt_amd import synthetic
    from mpi_opt_amd.gp import DeviceGP

    n, d, m, k = 200, 10, args.candidates, 5
    X, y = synthetic.gp_problem(n, d, 0)
    # hyper-parameters as fitted by sklearn on this data (tests/golden/gp_ei_n200_d10.npz)
    ls = np.array([16.2, 1.91, 1.65, 9.84, 1.84, 2.94, 2.45, 9.09, 8.13, 1.94])
    g = DeviceGP(X, y, 17.4955, ls, 0.0465, device=dev)
    cand = torch.from_numpy(synthetic.gp_candidates(m, d, seed=1 + rank)).to(dev)
    y_opt = float(np.min(y))
    torch.cuda.synchronize(dev)

    gathered = torch.empty(ws * 2, dtype=torch.float64, device=dev) if ws > 1 else None   # [rank][value, index]

    def step():
        out = g.score(cand, y_opt, acqs=("EI",), k=k, want_mu_sd=True, want_values=True)
        if ws > 1:
            idx, val = out["topk"]["EI"]
            local = torch.stack([val[0], (idx[0] + rank * m).to(torch.float64)])
            dist.all_gather_into_tensor(gathered, local)
        return out

    # W warmup steps, then the same step until >= 0.3 s of warmup has run: the GPU
    # clock ramps over the first ~30 ms of back-to-back launches (profiles/r01:
    # 2.0 -> 1.57 ms per launch), which a 3-step warmup does not cover.
    tw = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    while True:
        step()
        torch.cuda.synchronize(dev)
        # every rank must run the same number of steps (each holds an all-gather):
        # the ranks agree on whether any of them still needs warmup
        more = torch.tensor([1.0 if time.perf_counter() - tw < 0.3 else 0.0], dtype=torch.float64, device=dev)
        if ws > 1:
            dist.all_reduce(more, op=dist.ReduceOp.MAX)
        if float(more.item()) == 0.0:
            break
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

    # the ask step as a search pays it once per fitted model: the device
    # factorisation (DeviceGP: X / y to the device + mpo_gp_prepare) before the pass
    reps_p = 10
    torch.cuda.synchronize(dev)
    tp = time.perf_counter()
    for _ in range(reps_p):
        DeviceGP(X, y, 17.4955, ls, 0.0465, device=dev)
    torch.cuda.synchronize(dev)
    t_prep = (time.perf_counter() - tp) / reps_p

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
        "ask_step_ms": {"prepare": t_prep * 1e3, "score": dt / args.steps * 1e3,
                        "total": (t_prep + dt / args.steps) * 1e3,
                        "note": "prepare = DeviceGP construction (H2D of X, y + mpo_gp_prepare), once per "
                                "fitted model; value / ms_per_step time the scoring pass alone"},
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY §8d recipe: X~U[0,1]^{200x10}, y=sin(Xw)+0.1eps; candidates~U[0,1]^{1Mx10})",
        "config": {"workload": "BASELINE configs[1]: GP/EI ask step, 200 observations, 10-dim, "
                               f"{m} candidates per GPU, top-{k} (skopt argsort[:n_restarts])",
                   "n_obs": n, "dims": d, "candidates_per_gpu": m,
                   "parallelism": f"candidates sharded, {ws} GPU(s), all-gather of (value,index)"},
        "roofline": {"kernel": "gp_score_kernel (one acquisition pass, finish fused)", "bound": "mfma",
                     "achieved": achieved,
                     "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                     "frac_rocprof": _rocprof_frac(args, flops),
                     "kernel_ms_rocprof": _rocprof_ms(args),
                     "traffic": ((args.pmc or {}).get("ei") or {}).get("hbm_bytes_per_launch"),
                     "traffic_detail": (args.pmc or {}).get("ei"),
                     "kernel_ms": t_kernel * 1e3,
                     "algorithmic_flops_per_launch": flops,
                     "algorithmic_hbm_bytes_per_launch": algo_bytes,
                     "algorithmic_hbm_gbs": algo_bytes / t_kernel / 1e9},
    }
    return res


def _rocprof_ms(args):
    ns = ((args.pmc or {}).get("ei") or {}).get("rocprof_avg_ns")
    return ns / 1e6 if ns else None


def _rocprof_frac(args, flops):
    """The roofline fraction from rocprofv3's average gp_score_kernel duration (the
    figure profiles/ reproduces), beside the HIP-event ``frac``."""
    ms = _rocprof_ms(args)
    return flops / (ms / 1e3) / 1e12 / FP64_PEAK_TFLOPS if ms else None


def summary(res):
    """Compact per-leg figures, printed as the LAST key of the JSON line so that a
    stored tail of the line carries every leg (value, roofline fraction, MFMA busy,
    HBM traffic against the leg's floor)."""
    def r(x, nd=4):
        return None if x is None else round(float(x), nd)

    out = {}
    rf = res.get("roofline") or {}
    if res.get("metric", "").startswith("EI"):
        out["ei"] = {"value": r(res.get("value"), 0), "frac": r(rf.get("frac")), "frac_rocprof": r(rf.get("frac_rocprof")),
                     "kernel_ms_rocprof": r(rf.get("kernel_ms_rocprof")),
                     "traffic_MB": r((rf.get("traffic") or 0) / 1e6, 1) if rf.get("traffic") else None}
    for leg, floor_key in (("train", "every_tensor_once_hbm_bytes_per_train_batch"),
                           ("densenet", "every_tensor_once_hbm_bytes_per_train_step")):
        L = res.get(leg)
        if not L:
            continue
        lr = L.get("roofline") or {}
        pmc = lr.get("pmc") or {}
        tr, fl = lr.get("traffic"), lr.get(floor_key)
        out[leg] = {"value": r(L.get("value"), 1), "ms_per_step": r(L.get("ms_per_step"), 3), "frac": r(lr.get("frac")),
                    "mfma_busy": r(pmc.get("mfma_busy")), "traffic_GB": r(tr / 1e9 if tr else None, 2),
                    "traffic_vs_floor": r(tr / fl if tr and fl else None, 3)}
        if leg == "train" and L.get("shard_8gpu"):
            out[leg]["shard_factor"] = r(L["shard_8gpu"].get("factor"))
    if res.get("gp_fit"):
        out["gp_fit"] = {"value": r(res["gp_fit"].get("value"), 2), "unit": res["gp_fit"].get("unit")}
    if res.get("search"):
        out["search"] = {"told_per_h": r(res["search"].get("value"), 1),
                         "trained_per_h": r(res["search"].get("trained_per_hour"), 1)}
    if res.get("search_gp"):
        sg = res["search_gp"]
        proj = sg.get("projection_configs3_8gpu") or {}
        out["search_gp"] = {"told_per_h": r(sg.get("value"), 1),
                            "refits_per_optimizer_s": r(sg.get("refits_per_optimizer_s"), 1),
                            "ask256_ms_per_refit": r((sg.get("ask256") or {}).get("ms_per_refit"), 2),
                            "proj_8gpu_told_per_h": r(proj.get("told_trials_per_hour"), 1)}
    return out


def bench_gp_fit(args, torch, dev, cpu):
    """GP refit: skopt's L-BFGS-B hyper-parameter search with the
    LML + gradient on the device (all restarts batched per iteration), at the
    configs[1] problem (200 observations, D=10) -- and at n = 256 / 500, the sizes
    a 256-trial search reaches (real points + the cl_min lies of a batch ask).
    Rank 0 only: the optimizer runs on the coordinator rank.  CPU baseline:
    sklearn's own fit on the host cores (n = 200)."""
    from mpi_opt_amd import _lib, synthetic
    from mpi_opt_amd.gp_fit import DeviceLML, fit_lml, normalize_targets

    d = 10
    sizes = {}
    for n in (200, 256, 500):
        X, y = synthetic.gp_problem(n, d, 0)
        fit_lml(X, y, random_state=0, device=dev)                    # warm (allocation, first launch)
        reps = 2 if n > 256 else 3
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            _, det = fit_lml(X, y, random_state=0, device=dev, return_details=True)
        dt = (time.perf_counter() - t0) / reps
        lml = DeviceLML(X, normalize_targets(y)[0], device=dev)
        T = np.zeros((3, d + 2))
        lml.evaluate(T)
        stream = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            _lib.check(_lib.lib().mpo_gp_lml_grad(
                _lib.ptr(lml.X), _lib.ptr(lml.y), n, d, _lib.ptr(lml.theta_d), 3, _lib.ptr(lml.lml_d),
                _lib.ptr(lml.grad_d), _lib.ptr(lml.info_d), _lib.ptr(lml.ws), lml.ws_bytes, stream.cuda_stream))
        e1.record(stream)
        torch.cuda.synchronize(dev)
        sizes[n] = {"fits_per_s": 1.0 / dt, "ms_per_fit": dt * 1e3, "launches_per_fit": det["launches"],
                    "kernel_ms_per_launch": e0.elapsed_time(e1) / 10, "lml": det["lml"],
                    "kernel": "split block sweep" if n > 48 else "lml_grad_kernel (LDS Cholesky)"}
    s200 = sizes[200]
    out = {"metric": "GP refits/sec (skopt LML L-BFGS-B, 3 starts, N=200 obs, D=10, fp64)",
           "value": s200["fits_per_s"], "unit": "fits/s", "ms_per_fit": s200["ms_per_fit"],
           "launches_per_fit": s200["launches_per_fit"], "lml": s200["lml"], "dtype": "f64",
           "by_n": {str(k): v for k, v in sizes.items()},
           "kernel": {"name": "split block sweep (sw_xs_build, one sw_step per 32-wide pivot block, sw_alpha, "
                              "sw_pairs_final)", "ms_per_launch": s200["kernel_ms_per_launch"],
                      "thetas_per_launch": 3,
                      "note": "one LML evaluation of 3 thetas = one launch per 32-wide pivot block + 3; latency-"
                              "bound (the sequential pivot sweeps), not a roofline kernel"}}
    if cpu:
        from oracle import gp_ei as O

        X, y = synthetic.gp_problem(200, d, 0)
        t0 = time.perf_counter()
        st, gpr = O.fit_skopt_gp(X, y, random_state=0)
        t_cpu = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": 1.0 / t_cpu, "unit": "fits/s", "cores": host_cores(), "kind": "port",
                               "sample": f"one sklearn GaussianProcessRegressor.fit (the skopt refit) at n=200, "
                                         f"lml {gpr.log_marginal_likelihood_value_:.9f}, {t_cpu:.2f} s"}
    return out


def sample_trials(n, seed):
    """Trials drawn from the option3 mnist space (option3:127-131): nb_filters,
    pool_size, kernel_size, dense -- plus a per-trial Adam lr 10**U(-4,-2) and
    dropout rate U(0, 0.5), the configs[2] "ragged widths/lr/dropout" population
    (the reference's own dropout dimension is dead and trains at 0.25)."""
    from mpi_opt_amd.population import TrialSpec

    rng = np.random.RandomState(seed)
    out = []
    for i in range(n):
        F, p, k, dense = (int(rng.randint(10, 51)), int(rng.randint(2, 11)), int(rng.randint(2, 11)),
                          int(rng.randint(50, 201)))
        out.append(TrialSpec(nb_filters=F, pool_size=p, kernel_size=k, dense=dense,
                             lr=float(10.0 ** rng.uniform(-4, -2)), dropout=float(rng.uniform(0.0, 0.5)), seed=i))
    return out


def torch_cpu_trial_seconds(trials, concurrent=4, steps=3, val=1):
    """torch-CPU fp32 (oracle/cnn_torch.py) seconds per train step / validation
    batch of each trial at batch 100, ``concurrent`` trials at once on the host
    cores (cores // concurrent threads each; the -n 21 --block-size 5 layout)."""
    from oracle import cnn_torch as CT

    cores = host_cores()
    t0 = time.perf_counter()
    times, threads = CT.time_trials([(t.nb_filters, t.kernel_size, t.pool_size, t.dense) for t in trials],
                                    concurrent=concurrent, cores=cores, steps=steps, val=val, warmup=1)
    return times, cores, threads, time.perf_counter() - t0


def cpu_baseline_train(trials, n_sample=32, concurrent=4):
    """torch-CPU fp32 single-trial training (BASELINE.md:45-52), 4 trials at once
    with cores//4 threads each, timed on a bounded sample of steps of the first
    ``n_sample`` trials and extrapolated to whole trials (5-fold, 10 epochs, 60k
    samples: 24 000 train steps + 6 000 validation batches)."""
    sample = trials[:n_sample]
    times, cores, threads, wall = torch_cpu_trial_seconds(sample, concurrent)
    sec = [24000 * ts + 6000 * tv for ts, tv in times]
    value = concurrent * 3600.0 / float(np.mean(sec))
    return {"value": value, "unit": "trials/hour", "cores": cores, "kind": "port",
            "sample": f"torch-CPU fp32 restatement (oracle/cnn_torch.py): {len(sample)} of the trials, {concurrent} "
                      f"at once x {threads} threads, 3 train steps + 1 validation batch each (batch 100), "
                      f"extrapolated to 24000 train steps + 6000 validation batches per trial ({wall:.1f} s)"}


def _timed_train_steps(e, x, yl, order, torch, dev, steps=10):
    """ms per train step of engine ``e`` (2 untimed steps first)."""
    for s_ in range(2):
        e.train_step(x, yl, order, s_ * e.batch)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s_ in range(steps):
        e.train_step(x, yl, order, (s_ + 2) * e.batch)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / steps * 1e3


def shard_step_ratio(full_ms, members, folds, x, yl, otr, torch, dev, gpus=8, steps=10, batch=100):
    """ms per train step of one GPU's LPT share (by FLOPs, as DistributedEvaluator
    deals (trial, fold) units) of this population over ``gpus`` GPUs, against the
    whole population's ``full_ms``: how much of a population's training one of
    ``gpus`` GPUs still pays (small populations run at a higher per-member cost).
    The caller has dropped the whole population's engine first, as a rank of the
    8-GPU search holds only its own share: with the 320-member engine's buffers
    still resident the share measured 6.53 instead of 5.69 ms
    (scripts/shard_ratio_probe.py, profiles/r05/shard_ratio_probe.log)."""
    from mpi_opt_amd.blocks import lpt_assign
    from mpi_opt_amd.population import PopulationEngine

    owner = lpt_assign([m.flops_per_sample_train() for m in members], gpus)
    mine = [i for i, o in enumerate(owner) if o == 0]
    sub = PopulationEngine([members[i] for i in mine], batch=batch, device=dev)
    osub = otr[mine].contiguous()
    shard_ms = _timed_train_steps(sub, x, yl, osub, torch, dev, steps)
    del sub
    return {"gpus": gpus, "members": len(mine), "shard_ms_per_step": shard_ms, "full_ms_per_step": full_ms,
            "factor": shard_ms / full_ms, "note": "share timed alone (the whole population's engine freed first)"}


def bench_train(args, torch, dist, ws, rank, dev):
    from mpi_opt_amd.population import PopulationEngine, TrialSpec, kfold_split, synthetic_mnist

    n_trials, n_fold, B = args.train_trials, 5, 100
    trials = sample_trials(n_trials, seed=13579 + rank)
    members, folds = [], []
    for t in trials:
        for f in range(n_fold):
            members.append(TrialSpec(t.nb_filters, t.kernel_size, t.pool_size, t.dense, t.lr, t.dropout,
                                     seed=len(members)))
            folds.append(f)
    eng = PopulationEngine(members, batch=B, device=dev)
    x, yl = synthetic_mnist(60000, seed=rank, device=dev)
    tr = np.stack([kfold_split(60000, n_fold, f)[0] for f in folds])
    va = np.stack([kfold_split(60000, n_fold, f)[1] for f in folds])
    otr = torch.from_numpy(tr).to(dev)
    ova = torch.from_numpy(va).to(dev)
    steps_per_epoch, val_batches = tr.shape[1] // B, va.shape[1] // B   # 480, 120
    ratio = steps_per_epoch // val_batches                              # 4 train steps per val batch
    state = {"st": 0, "vb": 0}

    def macro_step():
        for _ in range(ratio):
            eng.train_step(x, yl, otr, (state["st"] % steps_per_epoch) * B)
            state["st"] += 1
        eng.eval_step(x, yl, ova, (state["vb"] % val_batches) * B)
        state["vb"] += 1

    for _ in range(args.train_warmup):
        macro_step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    stream = torch.cuda.current_stream(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.train_steps):
        macro_step()
    e1.record(stream)
    if ws > 1:   # the per-BO-round exchange: all-gather of per-(trial, fold) validation losses
        g = torch.empty(ws * len(members), dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(g, eng.val_loss_sum)
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t_gpu = e0.elapsed_time(e1) / 1e3
    if ws > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    t_macro = dt / args.train_steps
    macro_per_trial = steps_per_epoch // ratio * 10        # 120 macro-steps/epoch x 10 epochs
    trials_per_hour = ws * n_trials * 3600.0 / (t_macro * macro_per_trial)
    flops = (ratio * B * sum(m.flops_per_sample_train() for m in members)
             + B * sum(m.flops_per_sample_fwd() for m in members))
    achieved = flops / (t_gpu / args.train_steps) / 1e12
    # per train batch: the every-tensor-once floor, and each kernel's own minimum
    # (slabs of the deterministic split-K weight gradients and flip_w2's copies included)
    floor_bytes = sum(m.hbm_bytes_train(B) for m in members)
    by_kernel = collections.defaultdict(float)
    for m in members:
        for k, v in m.hbm_bytes_train_by_kernel(B).items():
            by_kernel[k] += v
    algo_bytes = sum(by_kernel.values())
    pmc = (args.pmc or {}).get("train") if n_trials == 64 else None
    shard = None
    if n_trials == 64 and ws == 1:
        full_ms = _timed_train_steps(eng, x, yl, otr, torch, dev)
        eng = None   # a rank of the 8-GPU search holds only its share: time it with the whole population freed
        gc.collect()
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        shard = shard_step_ratio(full_ms, members, folds, x, yl, otr, torch, dev, batch=B)
    if pmc and pmc.get("per_family_hbm_bytes"):
        fam = pmc["per_family_hbm_bytes"]
        pmc["per_family_vs_model"] = {k: {"measured": fam.get(k, 0.0), "model": v,
                                          "ratio": fam.get(k, 0.0) / v if v else None}
                                      for k, v in sorted(by_kernel.items(), key=lambda kv: -fam.get(kv[0], 0.0))}
    return {
        "metric": "MNIST-CNN trials/hour (5-fold CV, 10 epochs, 60k samples/trial-fold split)",
        "value": trials_per_hour, "unit": "trials/hour", "n_gpus": ws, "steps": args.train_steps,
        "warmup": args.train_warmup, "ms_per_step": t_macro * 1e3, "scaling": "weak", "dtype": "f32",
        "data": "synthetic MNIST-shape x~U[0,1] (60000x784 f32), uniform labels; glorot init",
        "config": {"workload": f"BASELINE configs[2]/[3]: {n_trials} ragged test_mnist trials x {n_fold} folds "
                               f"= {len(members)} population members per GPU; step = {ratio} train batches "
                               f"+ 1 validation batch (1/{steps_per_epoch // ratio} epoch)",
                   "trials_per_gpu": n_trials, "folds": n_fold, "batch": B, "epochs": 10,
                   "parallelism": f"trials sharded, {ws} GPU(s), all-gather of fold losses"},
        "roofline": {"kernel": "population step (all conv/dense MFMA kernels)", "bound": "mfma",
                     "achieved": achieved, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP32_PEAK_TFLOPS,
                     "traffic": pmc["hbm_bytes_per_train_batch"] if pmc else None,
                     "traffic_unit": "HBM bytes per train batch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, this run)",
                     "algorithmic_hbm_bytes_per_train_batch": algo_bytes,
                     "algorithmic_model": "per-kernel minimum (mpi_opt_amd.population.TrialSpec."
                                          "hbm_bytes_train_by_kernel)",
                     "every_tensor_once_hbm_bytes_per_train_batch": floor_bytes,
                     "algorithmic_flops_per_step": flops,
                     "pmc": pmc},
        "shard_8gpu": shard,
        "_trials": trials,
    }


def cpu_baseline_densenet(n_sample=4, concurrent=4):
    """torch-CPU fp32 DenseNet (oracle/densenet_torch.py, the reference grid
    architecture) at batch 100, 4 trials at once with cores//4 threads each:
    2 train steps + 1 validation batch per trial, extrapolated to a whole trial
    (10 epochs x (350 train + 150 validation batches))."""
    from oracle import densenet_torch as DT

    cores = host_cores()
    t0 = time.perf_counter()
    times, threads = DT.time_trials(n_sample, concurrent=concurrent, cores=cores, steps=2, val=1, warmup=1)
    wall = time.perf_counter() - t0
    sec = [10 * (350 * ts + 150 * tv) for ts, tv in times]
    return {"value": concurrent * 3600.0 / float(np.mean(sec)), "unit": "trials/hour", "cores": cores,
            "kind": "port",
            "sample": f"torch-CPU fp32 restatement (oracle/densenet_torch.py): {n_sample} trials, {concurrent} at once "
                      f"x {threads} threads, 2 train steps + 1 validation batch at batch 100 each, extrapolated to "
                      f"3500 train steps + 1500 validation batches per trial ({wall:.1f} s)"}


def bench_densenet(args, torch, dist, ws, rank, dev):
    """BASELINE config 5: a population of DenseNets (densenet.py, base_model.py grid:
    depth 10, 3 blocks, growth 12, nb_filter 16; lr = 10**U(-5, 1)) on synthetic
    CIFAR-10-shape data; each trial trains 10 epochs on the option3 70/30 split of
    50 000 samples (350 train + 150 validation batches of 100 per epoch)."""
    from mpi_opt_amd.densenet import DenseNetArch, DenseNetPopulation, flops_per_sample_fwd, \
        flops_per_sample_train, hbm_bytes_train, hbm_bytes_train_by_kernel, synthetic_cifar
    from mpi_opt_amd.population import kfold_split

    n_trials, B = args.dn_trials, 100
    rng = np.random.RandomState(2024 + rank)
    lrs = 10.0 ** rng.uniform(-5, 1, size=n_trials)
    pop = DenseNetPopulation(DenseNetArch(), lrs, batch=B, device=dev, init_seed=rank * 1000)
    x, yl = synthetic_cifar(50000, seed=rank, device=dev)
    tr, va = kfold_split(50000, 1, 0)
    otr = torch.from_numpy(np.stack([tr] * n_trials)).to(dev)
    ova = torch.from_numpy(np.stack([va] * n_trials)).to(dev)
    n_tr, n_va = len(tr) // B, len(va) // B        # 350, 150
    state = {"st": 0, "vb": 0}

    def macro_step():                               # 7 train + 3 validation batches = 1/50 epoch
        for _ in range(7):
            pop.train_step(x, yl, otr, (state["st"] % n_tr) * B)
            state["st"] += 1
        for _ in range(3):
            pop.eval_step(x, yl, ova, (state["vb"] % n_va) * B)
            state["vb"] += 1

    for _ in range(args.train_warmup):
        macro_step()
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    stream = torch.cuda.current_stream(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.train_steps):
        macro_step()
    e1.record(stream)
    if ws > 1:
        g = torch.empty(ws * n_trials, dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(g, pop.val_loss_sum)
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t_gpu = e0.elapsed_time(e1) / 1e3
    if ws > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    t_macro = dt / args.train_steps
    trials_per_hour = ws * n_trials * 3600.0 / (t_macro * 50 * 10)
    flops = n_trials * B * (7 * flops_per_sample_train(pop.layers) + 3 * flops_per_sample_fwd(pop.layers))
    achieved = flops / (t_gpu / args.train_steps) / 1e12
    # per train step: the every-tensor-once lower bound, and each kernel's own minimum
    # with the passes training-mode BatchNorm needs (statistics before use, reduce
    # before apply) -- the model the measured traffic is held against
    floor_bytes = n_trials * hbm_bytes_train(pop.layers, B, pop.n_params)
    by_kernel = {k: n_trials * v for k, v in hbm_bytes_train_by_kernel(pop.layers, B, pop.n_params).items()}
    algo_bytes = sum(by_kernel.values())
    pmc = (args.pmc or {}).get("densenet") if n_trials == 32 else None
    if pmc and pmc.get("per_family_hbm_bytes"):
        fam = pmc["per_family_hbm_bytes"]
        pmc["per_family_vs_model"] = {k: {"measured": fam.get(k, 0.0), "model": v,
                                          "ratio": fam.get(k, 0.0) / v if v else None}
                                      for k, v in sorted(by_kernel.items(), key=lambda kv: -fam.get(kv[0], 0.0))}
    return {
        "metric": "DenseNet trials/hour (CIFAR-10 shape, 10 epochs, 70/30 split of 50k samples)",
        "value": trials_per_hour, "unit": "trials/hour", "n_gpus": ws, "steps": args.train_steps,
        "warmup": args.train_warmup, "ms_per_step": t_macro * 1e3, "scaling": "weak", "dtype": "f32",
        "data": "synthetic CIFAR-10-shape x~U[0,1] (50000x32x32x3 f32), uniform labels; he_uniform init",
        "config": {"workload": f"BASELINE configs[4]: {n_trials} DenseNet trials (depth 10, 3 blocks, growth 12, "
                               f"nb_filter 16, lr 10**U(-5,1)) per GPU; step = 7 train + 3 validation batches "
                               f"(1/50 epoch)", "trials_per_gpu": n_trials, "batch": B, "epochs": 10,
                   "parallelism": f"trials sharded, {ws} GPU(s), all-gather of validation losses"},
        "roofline": {"kernel": "population step (all DenseNet kernels)", "bound": "mfma",
                     "achieved": achieved, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP32_PEAK_TFLOPS,
                     "traffic": pmc["hbm_bytes_per_train_step"] if pmc else None,
                     "traffic_unit": "HBM bytes per train step (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, this run)",
                     "algorithmic_hbm_bytes_per_train_step": algo_bytes,
                     "algorithmic_model": "per-kernel minimum incl. training-mode BatchNorm passes "
                                          "(mpi_opt_amd.densenet.hbm_bytes_train_by_kernel)",
                     "every_tensor_once_hbm_bytes_per_train_step": floor_bytes, "pmc": pmc,
                     "algorithmic_flops_per_step": flops},
    }


SEARCH_ARGV = ["--world-size", "21", "--block-size", "5", "--epochs", "10", "--num-iterations", "10",
               "--n-fold", "5", "--n-samples", "60000", "--synthetic-labels", "learnable"]


def bench_search(args, torch, dist, ws, rank, dev):
    """BASELINE configs[0], measured end to end: the option3 search
    ``-n 21 --block-size 5 --epochs 10 --num-iterations 10 --n-fold 5`` on 60k
    synthetic MNIST-shape samples, through the build's scheduler, the device
    Optimizer and the population engine (the in-flight tail is trained too, as
    the reference's blocks finish theirs).  Reports the measured trials/hour and
    the wall time split into optimizer (ask/tell) and training."""
    import tempfile

    from mpi_opt_amd import search

    a = search.make_parser().parse_args(SEARCH_ARGV + list(args.search_args or []))
    with tempfile.TemporaryDirectory() as tmp:
        a.checkpoint = os.path.join(tmp, "coordinator.pkl")
        # the scheduler polls blocks in random.shuffle order (unseeded in the reference,
        # coordinator.py:114), which decides which trials train and are told when: seeded
        # here so every bench run measures the same trials (scripts/search_repeat.py:
        # unseeded, two runs of this leg trained different trials, 30 s vs 51 s)
        random.seed(0)
        if ws > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        rep = search.run_search(a, log=lambda *m: print(*m, file=sys.stderr, flush=True))
        torch.cuda.synchronize(dev)
        if ws > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
    if rank != 0:
        return None
    out = {"metric": "MNIST-CNN trials/hour, measured search (BASELINE configs[0])",
           "value": rep["trials_told"] * 3600.0 / wall, "unit": "trials/hour (told)", "n_gpus": ws,
           "trained_per_hour": rep["trials_trained"] * 3600.0 / wall,
           "wall_s": wall, "scaling": "strong", "dtype": "f32",
           "config": {"workload": "option3 search " + " ".join(SEARCH_ARGV + list(args.search_args or [])),
                      "num_blocks": rep["num_blocks"], "populations": rep["populations"],
                      "parallelism": f"(trial, fold) units LPT-sharded over {ws} GPU(s)"},
           "trials_trained": rep["trials_trained"], "trials_told": rep["trials_told"],
           "split_s": {"optimizer_ask": rep["ask_s"], "optimizer_tell": rep["tell_s"],
                       "optimizer_chain_wait": rep["chain_wait_s"], "training": rep["train_s"],
                       "other": wall - rep["optimizer_s"] - rep["train_s"]},
           "asks": rep["asks"], "tells": rep["tells"], "best_fom": rep["best_fom"],
           "_trained_params": rep["trained_params"], "_num_blocks": rep["num_blocks"]}
    return out


# learnable synthetic labels (population.synthetic_mnist): with uniform labels every
# told FOM is the uniform-softmax BCE and the GP of the search fits a flat function
SEARCH3_ARGV = ["--world-size", "129", "--block-size", "2", "--n-fold", "5", "--num-iterations", "128",
                "--epochs", "1", "--n-samples", "60000", "--synthetic-labels", "learnable"]


def bench_search_gp(args, torch, dist, ws, rank, dev):
    """BASELINE configs[3]'s layout with the GP in the loop (the north_star search):
    64 blocks (``-n 129 --block-size 2``), 5-fold CV, cl_min batches of
    ``--num-iterations``.  Reduced to fit a bench run: 128 iterations instead of
    256 and 1 epoch instead of 10 (stated in ``config.workload``).  The first 64
    trials train as one population and are told one at a time; each of the
    following launches pays the reference's tell + ``ask(num_iterations)`` (a
    fresh cl_min batch after every fit, coordinator.py:46-50, 73) -- so the GP
    refits (one per tell and per lie) run between the two populations.  Then,
    on its own: ``Optimizer.ask(256)`` after 256 tells (the rank-0 term of the
    full 256-trial search while the GPUs train)."""
    import tempfile

    from mpi_opt_amd import optimizer as OPT
    from mpi_opt_amd import search
    from mpi_opt_amd.models import mnist_space

    argv = SEARCH3_ARGV + list(args.search3_args or [])
    a = search.make_parser().parse_args(argv)
    with tempfile.TemporaryDirectory() as tmp:
        a.checkpoint = os.path.join(tmp, "coordinator.pkl")
        # the scheduler polls blocks in random.shuffle order (unseeded in the reference,
        # coordinator.py:114), which decides which trials train and are told when: seeded
        # here so every bench run measures the same trials (scripts/search_repeat.py:
        # unseeded, two runs of this leg trained different trials, 30 s vs 51 s)
        random.seed(0)
        if ws > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        rep = search.run_search(a, log=lambda *m: print(*m, file=sys.stderr, flush=True))
        torch.cuda.synchronize(dev)
        if ws > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
    if rank != 0:
        return None
    gp = rep["gp"]
    samples = gp.pop("samples")
    opt_s = rep["optimizer_s"]
    out = {"metric": "MNIST-CNN trials/hour, measured search with the GP in the loop (BASELINE configs[3] layout)",
           "value": rep["trials_told"] * 3600.0 / wall, "unit": "trials/hour (told)", "n_gpus": ws,
           "wall_s": wall, "scaling": "strong", "dtype": "f32 training, f64 GP",
           "config": {"workload": "option3 search " + " ".join(argv) + " (configs[3]: -n 129 --block-size 2 "
                                  "--n-fold 5; reduced to 128 iterations and 1 epoch for the bench)",
                      "num_blocks": rep["num_blocks"], "populations": rep["populations"],
                      "parallelism": f"(trial, fold) units LPT-sharded over {ws} GPU(s); tells on rank 0; "
                                     f"cl_min ask batches LPT-dealt over {ws} GPU(s) x {rep['chain_workers']} "
                                     f"concurrent chains each"},
           "trials_told": rep["trials_told"], "trials_trained": rep["trials_trained"],
           "trained_per_hour": rep["trials_trained"] * 3600.0 / wall,
           "tail_trials": rep["tail_trials"],
           "split_s": {"optimizer_ask": rep["ask_s"], "optimizer_tell": rep["tell_s"],
                       "optimizer_chain_wait": rep["chain_wait_s"], "training": rep["train_s"],
                       "other": wall - opt_s - rep["train_s"]},
           "chain_workers": rep["chain_workers"], "chain_busy_s": rep["chain_busy_s"],
           "optimizer_share": opt_s / wall, "asks": rep["asks"], "tells": rep["tells"],
           "gp_refits": gp["refits"], "gp_refit_mean_n": gp["n_sum"] / max(1, gp["refits"]), "gp_refit_max_n": gp["n_max"],
           # refits completed per second of the search loop's optimizer time (tells + waiting on batches)
           "refits_per_optimizer_s": gp["refits"] / max(1e-9, opt_s),
           # per refit, summed over concurrent chains (worker-thread seconds, not wall)
           "ms_per_refit": 1e3 * gp["refit_s"] / max(1, gp["refits"]),
           "ms_per_proposal": 1e3 * gp["propose_s"] / max(1, gp["refits"]),
           "ms_per_proposal_split": {k: 1e3 * gp[k + "_s"] / max(1, gp["refits"]) for k in ("prepare", "score", "polish")},
           "best_fom": rep["best_fom"]}
    # the rank-0 Amdahl term of the full search: ask(256) after 256 tells
    rng = np.random.RandomState(256)
    opt = OPT.Optimizer(mnist_space(), random_state=13579, device=dev)
    pts = opt.space.rvs(n_samples=256, random_state=rng)
    ys = [float(((p[0] - 30) / 40) ** 2 + ((p[3] - 120) / 150) ** 2 + (p[4] - 0.3) ** 2 + 0.1 * rng.rand())
          for p in pts]
    opt.tell(pts[:-1], ys[:-1], fit=False)
    opt.tell(pts[-1], ys[-1])
    OPT.reset_stats()
    t0 = time.perf_counter()
    batch = opt.ask(args.ask_n)
    t_ask = time.perf_counter() - t0
    st = dict(OPT.STATS)
    out["ask256"] = {"n_points": args.ask_n, "told": 256, "seconds": t_ask, "refits": st["refits"],
                     "refit_n_range": [256, st["n_max"]], "ms_per_refit": 1e3 * st["refit_s"] / st["refits"],
                     "ms_per_proposal": 1e3 * st["propose_s"] / st["refits"],
                     "ms_per_proposal_split": {k: 1e3 * st[k + "_s"] / st["refits"] for k in ("prepare", "score", "polish")},
                     "distinct_points": len({tuple(b) for b in batch})}
    out["_told_state"] = (pts, ys)
    out["_samples"] = samples
    # the projection's inputs: this run's refits (n) and optimizer window, the sequential
    # ask(256)'s (n, seconds) latencies, the training GPU-seconds per 10-epoch 5-fold trial
    out["_proj"] = {"run_refit_ns": [n for n, _ in samples], "optimizer_s": opt_s,
                    "latency_samples": list(st["samples"]) + [sm for sm in samples if sm[0] < 64],
                    "trial_s_gpu": rep["train_s"] / max(1, rep["trials_trained"]) * 10.0,
                    "chain_workers": rep["chain_workers"]}
    out["timeline"] = rep["timeline"]
    return out


class _CountingOptimizer:
    """Stand-in optimizer that only counts the GP refits skopt's protocol runs (and
    at how many observations): a refit per tell once n_initial_points are told,
    and per ``ask(n, 'cl_min')`` the copy's refit plus one per lie."""

    def __init__(self, dimensions, random_state, n_initial_points=10, **_):
        self.rng = np.random.RandomState(random_state)
        self.dims = dimensions
        self.n0 = n_initial_points
        self.told = 0
        self.refits = []
        self.tell_refits = []        # the subset refitted by tells (rank 0, sequential)

    def _point(self):
        return [int(self.rng.randint(d.low, d.high + 1)) if type(d).__name__ == "Integer"
                else float(self.rng.uniform(d.low, d.high)) for d in self.dims]

    def tell(self, xs, ys):
        from mpi_opt_amd.optimizer import OptimizeResult

        self.told += len(ys)
        if self.told >= self.n0:
            self.refits.append(self.told)
            self.tell_refits.append(self.told)
        return OptimizeResult(x=list(xs[0]), fun=float(min(ys)))

    def ask(self, n):
        if self.told >= self.n0:
            self.refits.append(self.told)                      # copy(): re-tell, one refit
        self.refits.extend(self.told + i + 1 for i in range(n) if self.told + i + 1 >= self.n0)
        return [self._point() for _ in range(n)]


def protocol_refits(world_size, block_size, num_iterations, with_tells=False):
    """The refits (their observation counts) and populations the reference's
    protocol runs for an option3 layout: the build's scheduler and PopulationComm
    driven with instant random FOMs and a refit-counting optimizer (CPU only)."""
    import tempfile

    from mpi_opt_amd import scheduler as S
    from mpi_opt_amd.blocks import PopulationComm
    from mpi_opt_amd.models import mnist_space

    class _Instant:
        def __init__(self):
            self.rng = np.random.RandomState(0)

        def evaluate(self, params):
            return [float(v) for v in self.rng.rand(len(params))]

    nb = (world_size - 1) // block_size
    comm = PopulationComm(nb, block_size, _Instant())

    class _Sched(S.AskTellScheduler):
        optimizer_factory = staticmethod(lambda dims, rs, **kw: _CountingOptimizer(dims, rs))

    with tempfile.TemporaryDirectory() as tmp:
        sched = _Sched(comm, nb, mnist_space(), checkpoint=os.path.join(tmp, "c.pkl"))
        sched.run(num_iterations=num_iterations)
    if with_tells:
        return sched.optimizer.refits, list(comm.batches), sched.optimizer.tell_refits
    return sched.optimizer.refits, list(comm.batches)


def fit_refit_cost(samples, powers=(0, 1, 2)):
    """Non-negative least-squares t(n) = sum_p c_p n^p over measured (n, seconds)
    refit + proposal samples; returns [(p, c_p)].  Non-negative: a refit never gets
    cheaper with more observations, and a free fit through three noisy host samples
    gave a negative cubic term (t < 0 past n ~ 350) that under-priced the host path."""
    from scipy.optimize import nnls

    n = np.array([s[0] for s in samples], dtype=float)
    t = np.array([s[1] for s in samples], dtype=float)
    A = np.stack([n ** p for p in powers], 1)
    scale = np.abs(A).max(0)
    coef, _ = nnls(A / scale, t)
    return [(int(p), float(c / sc)) for p, c, sc in zip(powers, coef, scale)]


def _price(curve, ns):
    return float(sum(np.sum(c * ns ** p) for p, c in curve))


def project_configs3(proj, gpus=8, cpu=None, shard=None):
    """BASELINE configs[3] in full (``-n 129 --block-size 2 --n-fold 5
    --num-iterations 256 --epochs 10``, 256 trials over ``gpus`` GPUs), from this
    run's measured parts -- a projection, labelled as such (the 1-GPU full run
    itself is measured once per round: scripts/search_run.py, profiles/r04/):

    * the protocol's exact refit schedule (protocol_refits): the tells' refits on
      rank 0 one after another, each followed by an ask(256) chain of refits at
      n = told .. told + 255;
    * t(n): the sequential refit + proposal latency fitted on the standalone
      ask(256)'s refits and this run's small-n ones; ``scale`` = this run's
      optimizer window / sum of t over its refits (the measured concurrency of
      ``chain_workers`` chains on one GPU);
    * per population boundary, the chains over ``gpus`` GPUs: their work
      (sum t x scale) / gpus, but never below ceil(chains / (gpus x workers))
      rounds of one chain's latency under that concurrency (scale x workers x
      sum t over its refits);
    * training: trials x GPU-seconds per 10-epoch 5-fold trial x ``shard.factor``
      (one GPU's LPT share of a population vs the whole, measured in the train
      leg; 1 / gpus when absent).
    The optimizer and the populations do not overlap (a population's batches
    resolve before it trains)."""
    refits, pops, tells = protocol_refits(129, 2, 256, with_tells=True)
    coef = fit_refit_cost(proj["latency_samples"])
    ns = np.array(refits, dtype=float)
    run_ns = np.array(proj["run_refit_ns"], dtype=float)
    workers = max(1, int(proj.get("chain_workers") or 1))
    scale = proj["optimizer_s"] / max(1e-12, _price(coef, run_ns))
    t_tell = _price(coef, np.array(tells, dtype=float))
    t_chain, bounds, told = 0.0, [], 0
    for b, npop in enumerate(pops[:-1]):
        told += npop
        starts = np.arange(told - npop + 1, told + 1, dtype=float)      # told count at each ask of the boundary
        chain_seq = np.array([_price(coef, n0 + np.arange(256)) for n0 in starts])
        work = float(chain_seq.sum()) * scale / gpus
        floor = math.ceil(len(starts) / (gpus * workers)) * float(chain_seq.mean()) * scale * workers
        bounds.append({"chains": len(starts), "work_s": work, "latency_floor_s": floor, "seconds": max(work, floor)})
        t_chain += max(work, floor)
    trials = sum(pops)
    factor = shard["factor"] if shard else 1.0 / gpus
    t_train = trials * proj["trial_s_gpu"] * factor
    t_gp = t_tell + t_chain
    out = {"workload": "configs[3] in full: -n 129 --block-size 2 --n-fold 5 --num-iterations 256 --epochs 10, "
                       f"{gpus} GPUs (projection from this run's measured parts)",
           "refits": len(refits), "tell_refits": len(tells), "refit_n_mean": float(ns.mean()),
           "refit_n_max": int(ns.max()), "populations": pops, "trials_trained": trials,
           "trials_told": trials - pops[-1],
           "refit_latency_fit_s": coef, "chain_concurrency_scale": scale, "chain_workers": workers,
           "boundaries": bounds, "train_shard_factor": factor,
           "optimizer_s": t_gp, "optimizer_tells_s": t_tell, "optimizer_chains_s": t_chain, "training_s": t_train,
           "trials_per_hour": trials * 3600.0 / (t_gp + t_train),
           "told_trials_per_hour": (trials - pops[-1]) * 3600.0 / (t_gp + t_train),
           "optimizer_share": t_gp / (t_gp + t_train)}
    if cpu:
        ccoef = fit_refit_cost(cpu["samples"], powers=(2, 3))
        t_gp_cpu = _price(ccoef, ns)
        t_train_cpu = trials * cpu["trial_s"]
        out["cpu"] = {"refit_cost_fit_s": ccoef, "optimizer_s": t_gp_cpu, "training_s": t_train_cpu,
                      "trials_per_hour": trials * 3600.0 / (t_gp_cpu + t_train_cpu)}
        out["speedup_vs_cpu"] = out["trials_per_hour"] / out["cpu"]["trials_per_hour"]
    return out


def _oracle_refit_seconds(pts, ys, n):
    """Seconds of one skopt refit + proposal on the host at n observations (oracle:
    sklearn GaussianProcessRegressor.fit, einsum posterior over 10 000 candidates,
    scipy L-BFGS-B polish)."""
    from oracle.skopt_optimizer import SkoptOracle

    from mpi_opt_amd.models import mnist_space

    ora = SkoptOracle(mnist_space(), random_state=13579)
    ora.Xi, ora.yi = [list(p) for p in pts[:n]], list(ys[:n])
    ora._n_initial_points -= n
    t0 = time.perf_counter()
    ora._fit_and_propose()
    return time.perf_counter() - t0


def cpu_baseline_search_gp(out, cpu_train_trial_s):
    """The same search on the host the way the reference runs it, from bounded
    samples: the GP side is the oracle's skopt refit + proposal timed at three
    observation counts, fitted as a n^2 + b n^3 and summed over the run's refits;
    training is the torch-CPU restatement's per-trial time (the train leg's
    sample, 4 trials at once on every core) for the trials the run trained, at
    its epochs."""
    pts, ys = out.pop("_told_state")
    samples = [(n, _oracle_refit_seconds(pts, ys, n)) for n in (64, 160, 256)]
    coef = fit_refit_cost(samples, powers=(2, 3))
    ns = np.array([s_[0] for s_ in out.pop("_samples")], dtype=float)
    epochs = 1
    t_train = out["trials_trained"] * cpu_train_trial_s * epochs / 10.0
    t_gp = _price(coef, ns)
    t = t_gp + t_train
    res = {"value": out["trials_told"] * 3600.0 / t, "unit": "trials/hour (told)", "cores": host_cores(),
           "kind": "port", "seconds_gp": t_gp, "seconds_training": t_train,
           "refit_samples_s": [[n, t_] for n, t_ in samples], "refit_cost_fit_s": coef,
           "sample": f"GP: oracle skopt refit + proposal (sklearn GaussianProcessRegressor.fit, einsum posterior, "
                     f"L-BFGS-B polish, 10 000 candidates) timed once each at n = 64, 160, 256 "
                     f"({', '.join(f'{t_:.2f}' for _, t_ in samples)} s), fitted a n^2 + b n^3 and summed over the "
                     f"run's {len(ns)} refits; training: torch-CPU fp32 per-trial time of the train leg's sample "
                     f"({cpu_train_trial_s:.0f} s of all cores per 10-epoch 5-fold trial, 4 at once) x "
                     f"{out['trials_trained']} trials x {epochs}/10 epochs"}
    return res, {"samples": samples, "trial_s": cpu_train_trial_s}


def cpu_baseline_search(search_out, concurrent=4):
    """The same trials on the host the way the reference runs them: torch-CPU fp32
    single-trial training, ``num_blocks`` trials at once (cores // num_blocks
    threads each), launched in the search's order onto the first free block;
    per-trial time from a bounded sample of steps (3 train + 1 validation)."""
    from mpi_opt_amd.population import TrialSpec

    params = search_out.pop("_trained_params")
    nb = search_out.pop("_num_blocks")
    trials = [TrialSpec(nb_filters=int(p[0]), pool_size=int(p[1]), kernel_size=int(p[2]), dense=int(p[3]))
              for p in params]
    times, cores, threads, wall = torch_cpu_trial_seconds(trials, concurrent=nb)
    sec = [24000 * ts + 6000 * tv for ts, tv in times]
    free = [0.0] * nb
    for t in sec:                            # list schedule in launch order
        j = int(np.argmin(free))
        free[j] += t
    makespan = max(free)
    return {"value": len(trials) * 3600.0 / makespan, "unit": "trials/hour", "cores": cores, "kind": "port",
            "sample": f"the search's {len(trials)} trials, torch-CPU fp32 (oracle/cnn_torch.py), {nb} at once x "
                      f"{threads} threads, 3 train steps + 1 validation batch each, extrapolated to 24000 + 6000 "
                      f"per trial and list-scheduled onto {nb} blocks: makespan {makespan / 3600:.2f} h "
                      f"({wall:.1f} s); the GP is not reached (n_initial_points = 10)"}


def relaunch_distributed(n):
    """``bench.py --gpus N`` started without torch.distributed.run: start
    ``python -m torch.distributed.run --nproc-per-node N bench.py ...`` as a child
    process (one rank per GPU; this process never touches the GPU), pass its
    output through, return its exit code."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env={**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="all",
                    choices=["ei", "fit", "train", "densenet", "search", "search3", "all"])
    ap.add_argument("--search-args", nargs="*", default=None,
                    help="extra search CLI flags appended to configs[0]'s (e.g. --n-samples 6000)")
    ap.add_argument("--search3-args", nargs="*", default=None,
                    help="extra search CLI flags appended to the configs[3]-layout search's")
    ap.add_argument("--ask-n", type=int, default=256, help="cl_min batch size of the standalone ask after 256 tells")
    ap.add_argument("--candidates", type=int, default=1_000_000)
    ap.add_argument("--train-trials", type=int, default=64)
    ap.add_argument("--train-steps", type=int, default=5)
    ap.add_argument("--train-warmup", type=int, default=1)
    ap.add_argument("--dn-trials", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 traffic passes")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args.gpus))
    ws, rank, local = dist_env()
    args.pmc = None
    if ws == 1 and not args.no_pmc and args.workload in ("ei", "train", "densenet", "all") and shutil.which("rocprofv3"):
        t0 = time.perf_counter()
        args.pmc = live_pmc(args.train_trials)      # child processes, before this one touches the GPU
        args.pmc["wall_s"] = time.perf_counter() - t0
        for e in args.pmc["errors"]:
            print(f"warning: PMC pass failed: {e}", file=sys.stderr)

    import torch

    dist = None
    if ws > 1:
        import torch.distributed as dist

        # one rank per GPU over RCCL ("nccl").  MPO_BENCH_BACKEND=gloo with more ranks
        # than GPUs is a rehearsal of the N > 1 path on a one-GPU box only.
        backend = os.environ.get("MPO_BENCH_BACKEND", "nccl")
        local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    dev = torch.device("cuda", local if ws > 1 else 0)

    res = bench_ei(args, torch, dist, ws, rank, dev) if args.workload in ("ei", "all") else None
    fit = None
    if rank == 0 and args.workload in ("fit", "all"):
        fit = bench_gp_fit(args, torch, dev, ws == 1 and not args.no_cpu_baseline)
    train = bench_train(args, torch, dist, ws, rank, dev) if args.workload in ("train", "all") else None
    dn = bench_densenet(args, torch, dist, ws, rank, dev) if args.workload in ("densenet", "all") else None
    srch = bench_search(args, torch, dist, ws, rank, dev) if args.workload in ("search", "all") else None
    srch3 = bench_search_gp(args, torch, dist, ws, rank, dev) if args.workload in ("search3", "all") else None
    if rank == 0:
        cpu = ws == 1 and not args.no_cpu_baseline
        if srch is not None:
            if cpu:
                srch["cpu_baseline"] = cpu_baseline_search(srch)
            else:
                srch.pop("_trained_params")
                srch.pop("_num_blocks")
                srch["cpu_baseline"] = None
        if train is not None:
            trials = train.pop("_trials")
            train["cpu_baseline"] = cpu_baseline_train(trials) if cpu else None
        if srch3 is not None:
            cpu_parts = None
            if cpu:
                tcpu = (train or {}).get("cpu_baseline") or cpu_baseline_train(sample_trials(32, seed=13579))
                srch3["cpu_baseline"], cpu_parts = cpu_baseline_search_gp(srch3, 3600.0 / tcpu["value"])
            else:
                srch3.pop("_told_state")
                srch3.pop("_samples")
                srch3["cpu_baseline"] = None
            srch3["projection_configs3_8gpu"] = project_configs3(srch3.pop("_proj"), cpu=cpu_parts,
                                                                 shard=(train or {}).get("shard_8gpu"))
        if dn is not None:
            dn["cpu_baseline"] = cpu_baseline_densenet() if cpu else None
        if res is not None:
            res["cpu_baseline"] = cpu_baseline_ei() if cpu else None
            if fit is not None:
                res["gp_fit"] = fit
            if train is not None:
                res["train"] = train
            if dn is not None:
                res["densenet"] = dn
            if srch is not None:
                res["search"] = srch
            if srch3 is not None:
                res["search_gp"] = srch3
        else:
            res = next(r for r in (train, dn, srch, srch3, fit) if r is not None)
        res["summary"] = summary(res)      # last key: a stored tail of the line keeps every leg
        print(json.dumps(res), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
