"""The torch-CPU baseline trainer (oracle/cnn_torch.py) trains the same network
as the fp64 oracle (oracle/cnn.py): identical init, data order and dropout
masks give the same per-step loss trajectory (fp64 run: to 1e-10; the fp32
baseline as timed: within the north_star's 1e-3)."""
import numpy as np
import pytest
import torch

from oracle import cnn as C
from oracle import cnn_torch as T


@pytest.mark.parametrize("F,k,p,dense", [(10, 2, 2, 50), (17, 4, 3, 90), (12, 9, 5, 120)])
def test_torch_baseline_trajectory_matches_oracle(F, k, p, dense):
    rng = np.random.RandomState(3)
    x = rng.uniform(size=(40, 784)).astype(np.float32)
    y = rng.randint(0, 10, size=40)
    params = T.glorot_params(F, k, p, dense, seed=F)
    o = C.TrialOracle(F, k, p, dense, {n: v.astype(np.float64) for n, v in params.items()}, seed=5)
    masks = lambda step, layer, n, rate: C.dropout_keep(5, step, layer, n, rate)  # noqa: E731
    t64 = T.TorchTrial(F, k, p, dense, params, mask_fn=masks, dtype=torch.float64)
    t32 = T.TorchTrial(F, k, p, dense, params, mask_fn=masks)
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    for step in range(6):
        xb, yb = x[(step % 4) * 10:(step % 4) * 10 + 10], y[(step % 4) * 10:(step % 4) * 10 + 10]
        ref = o.train_step(xb, yb, step)
        sl = slice((step % 4) * 10, (step % 4) * 10 + 10)
        l64 = t64.train_step(xt[sl].double(), yt[sl], step)
        l32 = t32.train_step(xt[sl], yt[sl], step)
        assert abs(l64 - ref) <= 1e-10 * abs(ref), (step, l64, ref)
        assert abs(l32 - ref) <= 1e-3 * abs(ref), (step, l32, ref)


def test_time_trials_reports_positive_times():
    times, threads = T.time_trials([(10, 2, 2, 50), (12, 3, 3, 60)], concurrent=2, cores=2, steps=1, val=1,
                                   warmup=0)
    assert threads == 1 and len(times) == 2
    assert all(ts > 0 and tv > 0 for ts, tv in times)
