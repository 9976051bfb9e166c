import numpy as np
import pytest
import torch

from mpi_opt_amd.optimizer import Optimizer


def test_random_phase_and_result():
    opt = Optimizer([(10, 50), (0.0, 1.0)], n_initial_points=5, random_state=1)
    for i in range(4):
        x = opt.ask()
        assert 10 <= x[0] <= 50 and 0.0 <= x[1] <= 1.0
        r = opt.tell(x, float(i))
    assert r.fun == 0.0 and r.x == opt.Xi[0] and len(r.x_iters) == 4


def test_batch_ask_caches_until_tell():
    opt = Optimizer([(10, 50), (0.0, 1.0)], n_initial_points=100, random_state=2)
    a = opt.ask(3)
    assert opt.ask(3) is a and len(a) == 3
    opt.tell(a[0], 1.0)
    assert opt.ask(3) is not a


def test_seeded_sequences_are_reproducible():
    a = Optimizer([(10, 50), (2, 10), (0.0, 1.0)], random_state=13579)
    b = Optimizer([(10, 50), (2, 10), (0.0, 1.0)], random_state=13579)
    assert [a.ask() for _ in range(3)] == [b.ask() for _ in range(3)]


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_model_phase_fails_loudly_without_gpu():
    opt = Optimizer([(0.0, 1.0), (0.0, 1.0)], n_initial_points=3, random_state=0)
    X = [opt.ask() for _ in range(2)]
    opt.tell(X, [0.1, 0.2])
    with pytest.raises(Exception):
        opt.tell(opt.ask(), 0.3)   # third tell fits the GP: device-only, no CPU fallback
