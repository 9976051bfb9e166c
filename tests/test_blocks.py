import json
import math
import random

import pytest

from mpi_opt_amd.blocks import FOM_CEILING, PopulationComm, TrialEvaluator, lpt_assign
from mpi_opt_amd.models import BuilderFromFunction, mnist_space
from mpi_opt_amd.models import test_mnist as mnist_model_fn


class FakeEval:
    def __init__(self):
        self.calls = []

    def evaluate(self, params_list):
        self.calls.append([list(p) for p in params_list])
        return [sum(float(v) for v in p) / 1000.0 for p in params_list]


class StubOpt:
    def __init__(self):
        self.n = 0

    def ask(self, n):
        self.n += 1
        return [[self.n * 10 + i, 0.5] for i in range(n)]

    def tell(self, X, Y):
        class R:
            pass
        r = R()
        i = min(range(len(Y)), key=lambda j: Y[j])
        r.x, r.fun = X[i], Y[i]
        return r


def test_population_comm_drives_coordinator(tmp_path, monkeypatch):
    from mpi_opt_amd.scheduler import AskTellScheduler

    monkeypatch.chdir(tmp_path)

    class C(AskTellScheduler):
        optimizer_factory = staticmethod(lambda d, r: StubOpt())

        def save(self, fn=None):
            pass

    random.seed(0)
    ev = FakeEval()
    comm = PopulationComm(4, 5, ev)
    c = C(comm, 4, [(0, 1)])
    c.run(num_iterations=10)
    # launched blocks are trained together: the first batch holds all 4 blocks
    assert comm.batches[0] == 4
    # every trial launched is trained (the in-flight tail after the exit broadcast
    # too, as the reference's blocks finish theirs); only the told ones reach fom_list
    assert sum(comm.batches) == 10 == len(c.fom_list) + len(comm.results)
    assert comm.exited == set(range(1, 21))
    for p, f in zip(c.param_list, c.fom_list):
        assert f == sum(p) / 1000.0
    for p, f in comm.tail:
        assert f == sum(p) / 1000.0


@pytest.mark.parametrize("blocks,iters,seed", [(4, 10, 0), (4, 25, 1), (3, 17, 5), (8, 40, 2), (2, 9, 7)])
def test_population_width_is_kept(tmp_path, monkeypatch, blocks, iters, seed):
    """Ready results are collected before anything trains, so every population
    except the tail trained at the exit holds exactly ``num_blocks`` trials."""
    from mpi_opt_amd.scheduler import AskTellScheduler

    monkeypatch.chdir(tmp_path)

    class C(AskTellScheduler):
        optimizer_factory = staticmethod(lambda d, r: StubOpt())

        def save(self, fn=None):
            pass

    random.seed(seed)
    comm = PopulationComm(blocks, 2, FakeEval())
    c = C(comm, blocks, [(0, 1)])
    c.run(num_iterations=iters)
    assert sum(comm.batches) == iters
    assert all(b == blocks for b in comm.batches[:-1]), comm.batches
    assert 0 < comm.batches[-1] <= blocks
    told = len(c.fom_list)
    assert told == iters - blocks           # the reference leaves num_blocks trials untold


def test_lpt_balances():
    costs = [10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    owner = lpt_assign(costs, 3)
    loads = [sum(c for c, o in zip(costs, owner) if o == b) for b in range(3)]
    assert max(loads) - min(loads) <= 2


def test_foms_and_history_schema(tmp_path):
    ev = TrialEvaluator(BuilderFromFunction(mnist_model_fn, mnist_space()), None, None, n_fold=2,
                        history_dir=str(tmp_path))
    res = {(0, 0): {"val_loss": [0.5, 0.3], "val_acc": [0.1, 0.2]}, (0, 1): {"val_loss": [0.4, 0.1], "val_acc": [0, 0]},
           (1, 0): {"val_loss": [float("nan")], "val_acc": [0]}, (1, 1): {"val_loss": [0.2], "val_acc": [0]}}
    foms = ev.foms([[10, 2, 2, 50, 0.1], [20, 3, 3, 60, 0.2]], res)
    assert foms[0] == 0.2 and foms[1] == FOM_CEILING
    files = sorted(tmp_path.iterdir())
    assert len(files) == 4                  # one per (trial, fold), process_block.py:93-94
    docs = [json.loads(f.read_text()) for f in files]
    assert sorted(d["meta"]["fold"] for d in docs) == [0, 0, 1, 1]
    by = {(tuple(d["meta"]["parameters"]), d["meta"]["fold"]): d["history"]["0"] for d in docs}
    assert by[((10.0, 2.0, 2.0, 50.0, 0.1), 1)]["val_loss"] == [0.4, 0.1]
    assert all(list(d["history"]) == ["0"] for d in docs)
    assert math.isfinite(FOM_CEILING) and FOM_CEILING > 16


def test_units_carry_flops_and_folds():
    ev = TrialEvaluator(BuilderFromFunction(mnist_model_fn, mnist_space()), None, None, n_fold=3)
    u = ev.units([[10, 2, 2, 50, 0.1], [50, 2, 10, 200, 0.9]])
    assert [(t, f) for t, f, _, _ in u] == [(0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (1, 2)]
    assert u[3][3] > u[0][3]
