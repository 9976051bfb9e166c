"""--early-stopping / --target-metric (mpi_opt_amd.stopping): per-member rules
applied by the shared fold loop (population.train_folds), CPU only."""
import numpy as np
import pytest
import torch

from mpi_opt_amd.population import train_folds
from mpi_opt_amd.stopping import StopRule


def test_parse_forms():
    assert StopRule.from_args(None, None) is None
    r = StopRule.from_args("4")
    assert (r.patience, r.patience_metric, r.lower_is_better, r.target) == (4, "val_loss", True, None)
    r = StopRule.from_args("val_acc,~>,2", "val_loss,<=,0.1")
    assert (r.patience, r.patience_metric, r.lower_is_better) == (2, "val_acc", False)
    assert r.target == ("val_loss", "<=", 0.1)
    assert StopRule.from_args(None, "acc,>,0.9").target == ("val_acc", ">", 0.9)
    for bad in (("x", None), ("val_loss,<,3", None), ("-1", None), (None, "val_acc>0.9"), (None, "f1,>,0.5")):
        with pytest.raises(ValueError):
            StopRule.from_args(*bad)


def test_patience_is_keras_early_stopping():
    """Keras EarlyStopping(patience=N, min_delta=0): wait resets on a strictly
    better epoch, stops once N epochs in a row failed to improve."""
    st = StopRule.from_args("2").start(3)
    losses = [[1.0, 1.0, 1.0], [0.9, 1.0, 1.1], [0.9, 0.8, 1.2], [0.95, 0.9, 0.5], [0.7, 0.85, 0.6]]
    stops = [st.update(e, np.array(v), np.zeros(3)).tolist() for e, v in enumerate(losses)]
    # member 0: improves 0,1; no gain at 2, 3 -> stop after epoch 4 (index 3)
    # member 1: improves 0, 2; no gain at 1 (wait 1), 3, 4 -> stops at index 4
    # member 2: improves 0; fails 1, 2 -> stops at index 2
    assert stops == [[False] * 3, [False] * 3, [False, False, True], [True, False, False], [False, True, False]]
    assert st.epochs(5).tolist() == [4, 5, 3]
    st0 = StopRule.from_args("0").start(1)
    assert not st0.update(0, np.array([1.0]), np.zeros(1))[0]          # the first epoch always improves
    assert st0.update(1, np.array([1.0]), np.zeros(1))[0]


class _ScriptedEngine:
    """Stands in for a population: validation loss of member i after epoch e is
    script[i][e] (one validation batch of 1 sample); counts train steps."""

    def __init__(self, script):
        self.script = np.asarray(script, dtype=np.float32)
        self.n, self.batch, self.device = self.script.shape[0], 1, torch.device("cpu")
        self.val_loss_sum = torch.zeros(self.n)
        self.val_correct = torch.zeros(self.n, dtype=torch.int32)
        self.steps = 0
        self.epoch = -1

    def train_step(self, x, labels, order, row0):
        self.steps += 1
        return torch.zeros(self.n)

    def eval_reset(self):
        self.val_loss_sum.zero_()
        self.val_correct.zero_()
        self.epoch += 1

    def eval_step(self, x, labels, order, row0):
        self.val_loss_sum += torch.from_numpy(self.script[:, self.epoch])
        self.val_correct += (torch.from_numpy(self.script[:, self.epoch]) < 0.5).to(torch.int32)


def test_fold_loop_truncates_histories_and_stops_early():
    x = torch.zeros(10, 1)
    script = [[0.9, 0.8, 0.85, 0.86, 0.9], [0.9, 0.4, 0.3, 0.2, 0.1]]
    eng = _ScriptedEngine(script)
    rule = StopRule.from_args("2", "val_acc,>=,1")
    out = train_folds(eng, x, None, [0, 1], 2, 5, stopping=rule)
    # member 0 stops after epoch 4 (patience 2), member 1 at epoch 2 (acc 1 >= 1): loop ends at 4 of 5
    assert out["epochs_run"].tolist() == [4, 2]
    assert eng.epoch + 1 == 4 and eng.steps == 4 * 5    # 5 train samples per fold, batch 1
    eng2 = _ScriptedEngine(script)
    full = train_folds(eng2, x, None, [0, 1], 2, 5)
    assert full["epochs_run"].tolist() == [5, 5] and eng2.epoch + 1 == 5
    np.testing.assert_allclose(out["val_loss"][:, :4], full["val_loss"][:, :4])


def test_trial_fom_is_the_loss_at_the_stopping_epoch():
    from mpi_opt_amd.blocks import TrialEvaluator
    from mpi_opt_amd.models import BuilderFromFunction, mnist_space
    from mpi_opt_amd.models import test_mnist as fn

    ev = TrialEvaluator(BuilderFromFunction(fn, mnist_space()), None, None, n_fold=2)
    units = [(0, 0, None, 1.0), (0, 1, None, 1.0)]
    hist = {"val_loss": np.array([[0.5, 0.4, 0.45], [0.6, 0.3, 0.2]]), "val_acc": np.zeros((2, 3)),
            "epochs_run": np.array([2, 3])}
    res = ev._histories(units, hist)
    assert res[(0, 0)]["val_loss"] == [0.5, 0.4] and res[(0, 1)]["val_loss"] == [0.6, 0.3, 0.2]
    assert ev.foms([[10, 2, 2, 50, 0.1]], res) == [pytest.approx((0.4 + 0.2) / 2)]


def test_epoch_counts_are_pinned_for_every_form():
    """The stopping epochs each flag form gives on one scripted history (parity
    unpinned against mpi_learn; pinned here so the behaviour cannot drift)."""
    loss = np.array([[1.0, 0.9, 0.95, 0.96, 0.97, 0.5],
                     [1.0, 1.0, 1.0, 1.0, 1.0, 1.0],
                     [0.9, 0.8, 0.7, 0.6, 0.5, 0.4]])
    acc = np.array([[0.1, 0.5, 0.4, 0.4, 0.4, 0.9],
                    [0.2, 0.2, 0.3, 0.3, 0.3, 0.3],
                    [0.1, 0.2, 0.3, 0.96, 0.99, 0.99]])

    def epochs(es, tm):
        st = StopRule.from_args(es, tm).start(3)
        for e in range(loss.shape[1]):
            st.update(e, loss[:, e], acc[:, e])
        return st.epochs(loss.shape[1]).tolist()

    assert epochs("1", None) == [3, 2, 6]
    assert epochs("3", None) == [5, 4, 6]
    assert epochs("val_acc,~>,1", None) == [3, 2, 6]
    assert epochs("val_acc,~>,2", None) == [4, 5, 6]
    assert epochs(None, "val_acc,>,0.95") == [6, 6, 4]
    assert epochs(None, "val_loss,<=,0.6") == [6, 6, 4]
    assert epochs("2", "val_acc,>=,0.99") == [4, 3, 5]
