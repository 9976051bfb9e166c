"""Per-member stopping rules of fold training: option3's ``--early-stopping``
and ``--target-metric`` (/root/reference/hyperparameter_search_option3.py:66-69),
handed unchanged to mpi_learn's ``MPIKFoldManager(..., early_stopping=...,
target_metric=...)`` (/root/reference/process_block.py:83-90).

mpi_learn is un-vendored and unpinned, so this module's semantics
are **parity unpinned**: no fixture of the reference pins them.  The epoch
counts they produce are pinned by tests/test_stopping.py so that they cannot
change silently.  Its flags are restated as
the reference's help strings describe them, checked once per epoch after the
validation pass (the reference validates every epoch, option3:260):

* ``--early-stopping`` -- "patience for early stopping": ``N`` stops a member
  after N consecutive epochs without a strictly lower ``val_loss`` than its best
  so far (Keras ``EarlyStopping(patience=N)``, min_delta 0);
  ``METRIC,~<,N`` / ``METRIC,~>,N`` name the monitored metric (``val_loss`` or
  ``val_acc``) and whether lower or higher is better;
* ``--target-metric`` -- ``METRIC,OP,VALUE`` with OP one of ``<`` ``<=`` ``>``
  ``>=``: a member stops at the first epoch whose metric satisfies it.

A stopped member's history ends at its stopping epoch, so its figure of merit
(the last validation loss, averaged over folds) is the one at that epoch; the
population stops stepping once every member has stopped.
"""
from __future__ import annotations

import operator

import numpy as np

METRICS = ("val_loss", "val_acc")
_OPS = {"<": operator.lt, "<=": operator.le, ">": operator.gt, ">=": operator.ge}


def _metric(name, flag):
    name = name.strip()
    if name in ("loss", "acc"):
        name = "val_" + name
    if name not in METRICS:
        raise ValueError(f"{flag}: metric {name!r} is not one of {METRICS}")
    return name


class StopRule:
    """Parsed ``--early-stopping`` / ``--target-metric``; ``None`` when neither is set."""

    def __init__(self, patience=None, patience_metric="val_loss", lower_is_better=True, target=None):
        self.patience = patience
        self.patience_metric = patience_metric
        self.lower_is_better = lower_is_better
        self.target = target            # (metric, op symbol, value) or None

    @classmethod
    def from_args(cls, early_stopping=None, target_metric=None):
        if early_stopping in (None, "") and target_metric in (None, ""):
            return None
        rule = cls()
        if early_stopping not in (None, ""):
            parts = [p.strip() for p in str(early_stopping).split(",")]
            if len(parts) == 1:
                n = parts[0]
            elif len(parts) == 3 and parts[1] in ("~<", "~>"):
                rule.patience_metric = _metric(parts[0], "--early-stopping")
                rule.lower_is_better = parts[1] == "~<"
                n = parts[2]
            else:
                raise ValueError(f"--early-stopping {early_stopping!r}: expected N or METRIC,~<,N / METRIC,~>,N")
            try:
                rule.patience = int(n)
            except ValueError:
                raise ValueError(f"--early-stopping {early_stopping!r}: patience {n!r} is not an integer") from None
            if rule.patience < 0:
                raise ValueError(f"--early-stopping {early_stopping!r}: negative patience")
        if target_metric not in (None, ""):
            parts = [p.strip() for p in str(target_metric).split(",")]
            if len(parts) != 3 or parts[1] not in _OPS:
                raise ValueError(f"--target-metric {target_metric!r}: expected METRIC,OP,VALUE with OP in {list(_OPS)}")
            try:
                value = float(parts[2])
            except ValueError:
                raise ValueError(f"--target-metric {target_metric!r}: {parts[2]!r} is not a number") from None
            rule.target = (_metric(parts[0], "--target-metric"), parts[1], value)
        return rule

    def start(self, n_members):
        return StopState(self, n_members)


class StopState:
    """The rule applied to one population's members, epoch by epoch."""

    def __init__(self, rule, n):
        self.rule = rule
        self.stopped = np.zeros(n, dtype=bool)
        self.best = np.full(n, np.inf if rule.lower_is_better else -np.inf)
        self.since = np.zeros(n, dtype=np.int64)
        self.stop_epoch = np.zeros(n, dtype=np.int64)

    def update(self, epoch, val_loss, val_acc):
        """After epoch ``epoch`` (0-based): returns the members that stop now."""
        r = self.rule
        vals = {"val_loss": np.asarray(val_loss, dtype=np.float64), "val_acc": np.asarray(val_acc, dtype=np.float64)}
        now = np.zeros_like(self.stopped)
        if r.patience is not None:
            v = vals[r.patience_metric]
            better = v < self.best if r.lower_is_better else v > self.best
            self.best = np.where(better, v, self.best)
            self.since = np.where(better, 0, self.since + 1)
            now |= ~better & (self.since >= r.patience)      # Keras: wait >= patience on a non-improving epoch
        if r.target is not None:
            name, op, value = r.target
            now |= _OPS[op](vals[name], value)
        now &= ~self.stopped
        self.stopped |= now
        self.stop_epoch[now] = epoch + 1
        return now

    def all_stopped(self):
        return bool(self.stopped.all())

    def epochs(self, epochs):
        """Epochs each member's history keeps."""
        return np.where(self.stopped, self.stop_epoch, epochs)
