"""The refit schedule the reference's protocol implies (bench.protocol_refits):
the build's scheduler + PopulationComm driven with instant FOMs and a
refit-counting optimizer.  The counting rule is skopt's (a refit per tell once
n_initial_points = 10 are told; per ask(n, "cl_min") the copy's refit plus one
per lie, coordinator.py:46-50 / 63-79) -- the same rule the device Optimizer
follows (17 refits for 20 tells + ask(5) in tests/test_optimizer_parity_gpu.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_configs0_and_configs3_refit_schedules():
    import bench

    refits, pops = bench.protocol_refits(21, 5, 10)          # configs[0]: -n 21 --block-size 5, 10 iterations
    assert pops == [4, 4, 2] and len(refits) == 21 and min(refits) == 10
    refits, pops = bench.protocol_refits(129, 2, 128)        # configs[3] layout, 128 iterations
    assert pops == [64, 64] and len(refits) == 8255 and max(refits) == 191


def test_counting_optimizer_matches_the_device_rule():
    import bench
    from mpi_opt_amd.models import mnist_space

    o = bench._CountingOptimizer(mnist_space(), 0)
    for i in range(20):
        o.tell([o._point()], [float(i)])
    assert len(o.refits) == 11                              # tells 10 .. 20
    o.ask(5)
    assert len(o.refits) == 17 and o.refits[11:] == [20, 21, 22, 23, 24, 25]


def test_refit_cost_fit_recovers_a_polynomial():
    import numpy as np

    import bench

    samples = [(n, 0.002 + 1e-5 * n + 3e-8 * n * n) for n in range(10, 500, 7)]
    coef = dict(bench.fit_refit_cost(samples))
    assert np.allclose([coef[0], coef[1], coef[2]], [0.002, 1e-5, 3e-8], rtol=1e-6)


def test_configs3_projection_splits_tells_and_chains():
    """project_configs3: tell refits cost their sequential latency on rank 0; chain
    refits cost their measured concurrent share, divided over the GPUs."""
    import bench

    refits, pops, tells = bench.protocol_refits(129, 2, 256, with_tells=True)
    assert len(refits) == 49471 and pops == [64, 64, 64, 64] and len(tells) == 182
    proj = {"run_refit_ns": [100] * 1000, "optimizer_s": 10.0, "trial_s_gpu": 3.0, "chain_workers": 4,
            "latency_samples": [(n, 0.01) for n in range(10, 500, 10)]}            # flat 10 ms latency
    p8, p1 = bench.project_configs3(proj, gpus=8), bench.project_configs3(proj, gpus=1)
    assert abs(p8["optimizer_tells_s"] - 182 * 0.01) < 1e-9 and p1["optimizer_tells_s"] == p8["optimizer_tells_s"]
    # chains: 3 boundaries x 64 ask(256) chains x 256 refits x 10 ms (measured as 10 s per 1000
    # refits at 4 workers: scale 1), / gpus; the latency floor (ceil(64 / (gpus x 4)) rounds of
    # a 256-refit chain running 4x slower under 4-way sharing) meets the work bound exactly here
    assert abs(p1["optimizer_chains_s"] - 3 * 64 * 256 * 0.01) < 1e-6
    assert abs(p8["optimizer_chains_s"] * 8 - p1["optimizer_chains_s"]) < 1e-6
    assert all(abs(b["work_s"] - b["latency_floor_s"]) < 1e-9 for b in p8["boundaries"])
    assert abs(p8["training_s"] - 256 * 3.0 / 8) < 1e-9
    # one GPU's share of a population measured at 0.2 of the whole (not 1/8)
    ps = bench.project_configs3(proj, gpus=8, shard={"factor": 0.2})
    assert abs(ps["training_s"] - 256 * 3.0 * 0.2) < 1e-9
    # 32 GPUs x 4 workers = 128 slots for 64 chains: one chain's latency bounds each boundary
    p32 = bench.project_configs3(proj, gpus=32)
    assert all(b["seconds"] == b["latency_floor_s"] > b["work_s"] for b in p32["boundaries"])
