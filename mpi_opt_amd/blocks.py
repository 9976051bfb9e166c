"""Trial evaluation: the replacement for ProcessBlock + mpi_learn.

Reference (/root/reference/process_block.py:9-121): every block of MPI ranks
loops barrier -> recv params from rank 0 -> build the Keras model ->
``MPIKFoldManager(...).train()`` -> ``figure_of_merit()`` -> record details ->
``isend`` the FOM to rank 0.  Here:

* :class:`TrialEvaluator` trains a *batch* of trials x folds as one device
  population (:class:`~mpi_opt_amd.population.PopulationEngine`) and returns one
  FOM per trial: the fold-averaged validation loss after the last epoch (the
  ``hist["history"]["0"]["val_loss"][-1]`` convention of option0:71-82),
  non-finite losses clamped to the clipped-BCE ceiling 16.12 (a diverged trial
  must never hang or poison the GP);
* :class:`PopulationComm` is an MPI-communicator stand-in for the reference's
  unchanged ``Coordinator`` (coordinator.py:7-150) or this build's
  :class:`~mpi_opt_amd.scheduler.AskTellScheduler`: ``send`` records the
  parameters each rank of a block receives (tag 4), ``irecv`` from a block
  master returns a request whose ``test()`` answers "not done" while some block
  is still idle or another block's result is waiting to be collected and, once
  every block is busy and nothing is waiting, trains all launched blocks
  together -- the blocks the reference runs concurrently on MPI ranks run
  concurrently as population members on the GPU.  After the exit broadcast
  (``send(None)``) the ``Barrier`` trains the trials still in flight, as the
  reference's blocks finish theirs before reading the exit message
  (process_block.py:104-121); their FOMs are never told (coordinator.py:98-101);
* :class:`DistributedEvaluator` shards (trial, fold) units over the ranks of a
  torch.distributed group (RCCL over xGMI) by longest-processing-time on the
  per-unit FLOPs, with no data-path collective: rank 0 broadcasts the batch of
  suggestions, every rank trains its shard, the per-unit FOMs are all-gathered.
"""
from __future__ import annotations

import hashlib
import json
import math
import os
import types

import numpy as np

from .chains import LazyPoint, resolve, resolve_all
from .tag_lookup import tag_lookup

FOM_CEILING = -math.log(1e-7)   # clipped binary cross-entropy cannot exceed this


def lpt_assign(costs, n_bins):
    """Longest-processing-time-first: returns bin index per item."""
    order = sorted(range(len(costs)), key=lambda i: -costs[i])
    load = [0.0] * n_bins
    out = [0] * len(costs)
    for i in order:
        b = min(range(n_bins), key=lambda j: (load[j], j))
        out[i] = b
        load[b] += costs[i]
    return out


class TrialEvaluator:
    """Trains trials (parameter lists of ``model_provider``'s space) on one GPU."""

    def __init__(self, model_provider, x, y, n_fold=1, epochs=10, batch=100, lr=1e-3, device=None,
                 history_dir=None, init_seed=0, holdout=None, progress=None, loss="binary_crossentropy",
                 optimizer="adam", stopping=None):
        self.model_provider = model_provider
        self.x, self.y = x, y
        self.n_fold, self.epochs, self.batch, self.lr = n_fold, epochs, batch, lr
        # option3 --loss / --optimizer (hyperparameter_search_option3.py:60-61, Algo :270-275) for the
        # test_mnist populations; DenseNet trials train as their builder compiles them
        # (categorical_crossentropy + Adam, base_model.py:71-72)
        self.loss, self.optimizer = loss, optimizer
        self.stopping = stopping    # stopping.StopRule: --early-stopping / --target-metric (process_block.py:83-90)
        self.device = device
        self.history_dir = history_dir
        self.init_seed = init_seed
        self.holdout = holdout      # training samples of the train_list files (None: 70 % of x)
        self.n_evaluated = 0
        self.train_s = 0.0          # wall seconds spent training populations (synchronised)
        self.progress = progress    # callable(str): a line per trained epoch (long runs)

    def units(self, params_list):
        """(trial index, fold) pairs with their training FLOPs (LPT cost)."""
        out = []
        folds = max(1, self.n_fold)
        for t, params in enumerate(params_list):
            spec = self.model_provider.builder(*params).spec(lr=self.lr)
            cost = spec.flops_per_sample_train()
            for f in range(folds):
                out.append((t, f, spec, cost))
        return out

    def train_units(self, units, seed_base=0, trial_ids=None):
        """Train the given (trial, fold, spec) units as populations -- one for the
        test_mnist units, one per DenseNet architecture; returns
        {(trial, fold): history dict}.  Trial ``t`` is seeded by its identity
        ``trial_ids[t]`` (default ``seed_base + t``)."""
        import time

        t0 = time.perf_counter()
        tid = (lambda t: seed_base + t) if trial_ids is None else (lambda t: int(trial_ids[t]))
        try:
            return self._train_units(units, tid)
        finally:
            self.train_s += time.perf_counter() - t0

    def _train_units(self, units, tid):
        from .models import DenseNetSpec

        out = {}
        mnist = [u for u in units if not isinstance(u[2], DenseNetSpec)]
        out.update(self._train_mnist(mnist, tid))
        groups = {}
        for u in units:
            if isinstance(u[2], DenseNetSpec):
                groups.setdefault(u[2].arch.key(), []).append(u)
        for us in groups.values():
            out.update(self._train_densenet(us, tid))
        return out

    def _uid(self, trial_id, f):
        # seeds depend on the unit's identity only, never on how units are
        # sharded, batched or chunked: results are independent of the world size
        return (self.init_seed + 1000003 * trial_id + f) & 0x7FFFFFFF

    def _train_mnist(self, units, tid):
        from .population import PopulationEngine, TrialSpec, glorot_uniform_init

        if not units:
            return {}
        specs, folds, init = [], [], []
        for (t, f, spec, _) in units:
            uid = self._uid(tid(t), f)
            s = TrialSpec(spec.nb_filters, spec.kernel_size, spec.pool_size, spec.dense, spec.lr, spec.dropout,
                          seed=uid, loss=self.loss, optimizer=self.optimizer)
            specs.append(s)
            folds.append(f)
            init.append(glorot_uniform_init(s, uid))
        eng = PopulationEngine(specs, batch=self.batch, device=self.device, init=init)
        return self._histories(units, eng.fit_folds(self.x, self.y, folds, self.n_fold, self.epochs,
                                                      holdout=self.holdout, progress=self._epoch_cb(len(units)),
                                                      stopping=self.stopping))

    def _epoch_cb(self, members):
        if self.progress is None:
            return None
        import time

        t0 = time.perf_counter()
        return lambda ep, eps: self.progress(f"population of {members} members: epoch {ep}/{eps} "
                                             f"({time.perf_counter() - t0:.1f} s)")

    def _train_densenet(self, units, tid):
        from .densenet import DenseNetPopulation, he_uniform_init

        arch = units[0][2].arch
        layers = arch.layers()
        lrs = [u[2].lr for u in units]
        folds = [u[1] for u in units]
        init = [he_uniform_init(layers, self._uid(tid(t), f)) for (t, f, _, _) in units]
        pop = DenseNetPopulation(arch, lrs, batch=self.batch, device=self.device, init=init)
        return self._histories(units, pop.fit_folds(self.x, self.y, folds, self.n_fold, self.epochs,
                                                      holdout=self.holdout, progress=self._epoch_cb(len(units)),
                                                      stopping=self.stopping))

    @staticmethod
    def _histories(units, hist):
        out = {}
        for i, (t, f, _, _) in enumerate(units):
            e = int(hist["epochs_run"][i])         # a stopped member's history ends at its stopping epoch
            out[(t, f)] = {"val_loss": [float(v) for v in hist["val_loss"][i][:e]],
                           "val_acc": [float(v) for v in hist["val_acc"][i][:e]]}
            for key in ("dropped_train_samples", "dropped_val_samples"):
                if key in hist:
                    out[(t, f)][key] = int(hist[key][i])
        return out

    def foms(self, params_list, results):
        folds = max(1, self.n_fold)
        foms = []
        for t, params in enumerate(params_list):
            vals = [results[(t, f)]["val_loss"][-1] for f in range(folds)]
            fom = float(np.mean(vals))
            if not math.isfinite(fom):
                fom = FOM_CEILING
            foms.append(fom)
            self._record(params, [results[(t, f)] for f in range(folds)])
        return foms

    accepts_trial_ids = True

    def evaluate(self, params_list, trial_ids=None):
        """FOMs of ``params_list``; trial ``t`` is seeded by ``trial_ids[t]``
        (default: its position in the sequence of evaluated trials)."""
        units = self.units(params_list)
        if trial_ids is None:
            results = self.train_units(units, seed_base=self.n_evaluated)
        else:
            results = self.train_units(units, seed_base=self.n_evaluated, trial_ids=trial_ids)
        self.n_evaluated += len(params_list)
        return self.foms(params_list, results)

    def _record(self, params, fold_hists):
        """History JSON per (trial, fold) in the schema option0/1 parse
        (``history["0"]["val_loss"]``, option0:71-82): each fold's manager records
        its own details with ``meta = {"parameters": ..., "fold": manager.fold_num}``
        (process_block.py:93-94), so one file per fold, ``fold`` = its index."""
        if not self.history_dir:
            return
        os.makedirs(self.history_dir, exist_ok=True)
        h = hashlib.md5(json.dumps([float(p) if not isinstance(p, str) else p for p in params]).encode()).hexdigest()
        for fold, fh in enumerate(fold_hists):
            doc = {"history": {"0": fh}, "meta": {"parameters": [float(p) for p in params], "fold": fold}}
            with open(os.path.join(self.history_dir, f"{h}_fold{fold}.json"), "w") as f:
                json.dump(doc, f)


def _same_params(a, b):
    if isinstance(a, LazyPoint) or isinstance(b, LazyPoint):
        return a is b
    return a == b


class _Request:
    def __init__(self, comm, block):
        self.comm, self.block = comm, block

    def test(self):
        c = self.comm
        if self.block not in c.results:
            if c.results:
                return False, None      # other results are waiting: let the scheduler collect them first
            if len(c.busy) < c.num_blocks:
                return False, None      # another block is idle: let the scheduler fill it first
            c.evaluate_pending()        # every block busy, nothing ready: train the launched blocks together
        c.busy.discard(self.block)
        return True, c.results.pop(self.block)


def _batch_seq(p):
    """Submission number of a lazy point's ask batch (-1: already a plain point)."""
    return p.batch.seq if isinstance(p, LazyPoint) and p.batch.seq is not None else -1


class PopulationComm:
    """MPI-communicator stand-in for :class:`Coordinator` (size = 1 + blocks x block_size)."""

    def __init__(self, num_blocks, block_size, evaluator, train_tail=True, chunks=1):
        self.num_blocks, self.block_size, self.evaluator = num_blocks, block_size, evaluator
        self.train_tail = train_tail
        # chunks > 1: a population trains in that many parts, each as soon as its own
        # lazy ask batches resolve, so the later batches run while the earlier parts
        # train.  A member's training does not depend on its population (bit-identical
        # alone or in any population), so FOMs, tells and asks are unchanged.
        self.chunks = max(1, int(chunks))
        self.received = {}       # rank -> last params
        self.pending = {}        # block -> params launched, not yet trained
        self.results = {}        # block -> fom
        self.exited = set()
        self.busy = set()        # launched blocks whose result has not been collected
        self.batches = []        # sizes of the populations trained
        self.trained_params = [] # parameters of every trial trained, in training order
        self.tail = []           # (params, fom) of trials trained after the exit broadcast (never told)
        # per population: (seconds since the previous population finished, seconds waiting for
        # its lazy ask batches, seconds training it, trials) -- the search's timeline
        self.timeline = []
        self.on_population = None   # optional callback(index, timeline entry) after each population
        import time

        self._t_last = time.perf_counter()

    def Get_size(self):
        return 1 + self.num_blocks * self.block_size

    def Get_rank(self):
        return 0

    def _block_of(self, rank):
        return (rank - 1) // self.block_size + 1

    def send(self, obj, dest, tag):
        if tag != tag_lookup("params"):
            raise ValueError(f"unexpected tag {tag}")
        if obj is None:
            self.exited.add(dest)
            return
        # a point of a lazy ask batch (mpi_opt_amd.chains) stays unresolved until
        # its population trains: the same object must reach every rank of the block
        val = obj if isinstance(obj, LazyPoint) else list(obj)
        self.received[dest] = val
        b = self._block_of(dest)
        first = (b - 1) * self.block_size + 1
        ranks = range(first, first + self.block_size)
        if all(_same_params(self.received.get(r), val) for r in ranks):
            self.pending[b] = val
            self.busy.add(b)

    def irecv(self, source, tag):
        if tag != tag_lookup("result"):
            raise ValueError(f"unexpected tag {tag}")
        return _Request(self, self._block_of(source))

    def evaluate_pending(self):
        import time

        t0 = time.perf_counter()
        blocks = sorted(self.pending)
        points = [self.pending.pop(b) for b in blocks]
        k = min(self.chunks, len(points))
        # a trial's seed identity is its population's base plus its block-order
        # position, whatever part it trains in (evaluators that seed trials)
        base = self.trials_trained
        # parts in the order their ask batches were submitted (the executors run them
        # first-in first-out; the scheduler polls blocks in a shuffled order, so block
        # order is not submission order); results go back to their blocks
        order = sorted(range(len(points)), key=lambda i: (_batch_seq(points[i]), i)) if k > 1 else \
            list(range(len(points)))
        cuts = [len(points) * i // k for i in range(k + 1)]
        params, foms, wait = [None] * len(points), [None] * len(points), 0.0
        for c0, c1 in zip(cuts[:-1], cuts[1:]):
            idx = order[c0:c1]
            tw = time.perf_counter()
            part = resolve_all([points[i] for i in idx])
            wait += time.perf_counter() - tw
            if getattr(self.evaluator, "accepts_trial_ids", False):
                got = self.evaluator.evaluate(part, trial_ids=[base + i for i in idx])
            else:
                got = self.evaluator.evaluate(part)
            for i, p_, f_ in zip(idx, part, got):
                params[i], foms[i] = p_, f_
        t2 = time.perf_counter()
        t1 = t0 + wait
        self.timeline.append((t0 - self._t_last, wait, t2 - t1, len(params)))
        self._t_last = t2
        if self.on_population is not None:
            self.on_population(len(self.timeline) - 1, self.timeline[-1])
        self.batches.append(len(params))
        self.trained_params.extend(params)
        for b, f in zip(blocks, foms):
            self.results[b] = f

    def Barrier(self):
        if self.train_tail and self.exited and self.pending:
            # the points stay lazy here too: evaluate_pending resolves them (by chunk)
            launched = dict(self.pending)
            self.evaluate_pending()
            self.tail = [(resolve(launched[b]), self.results[b]) for b in sorted(launched)]

    @property
    def trials_trained(self):
        return sum(self.batches)


def local_topk(payload, s0, s1, device=None):
    """Score candidates [s0, s1) of a sharded acquisition request on this rank's
    GPU; returns {acq: (values, global indices)} of the shard's lowest-index-first
    top-k (skopt's ``np.argsort(values)[:k]`` restricted to the shard)."""
    from .optimizer import GPModel

    p = payload
    k = min(int(p["k"]), s1 - s0)
    est = GPModel(p["Xt"], p["y"], p["amp"], p["ls"], p["noise"], device=device)
    top = _device_topk(est, p["cand"][s0:s1], p["y_opt"], tuple(p["acqs"]), p["xi"], p["kappa"], k)
    return {a: (v, i + s0) for a, (v, i) in top.items()}


def _device_topk(est, X, y_opt, acqs, xi, kappa, k):
    import torch

    from . import _lib

    if k <= _lib.MPO_TOPK_MAX:
        sc = est.dev.score(X, y_opt, acqs=acqs, xi=xi, kappa=kappa, k=k, want_mu_sd=False, want_values=False)
        return {a: (sc["topk"][a][1].cpu().numpy(), sc["topk"][a][0].cpu().numpy()) for a in acqs}
    sc = est.dev.score(X, y_opt, acqs=acqs, xi=xi, kappa=kappa, k=0, want_mu_sd=False, want_values=True)
    out = {}
    for a in acqs:
        v, i = torch.sort(sc["values"][a], stable=True)
        out[a] = (v[:k].cpu().numpy(), i[:k].cpu().numpy())
    return out


def merge_topk(parts, k):
    """Global lowest-index-first top-k from per-shard lists [(values, indices)]:
    lexicographic (value, index), exactly the single-device order."""
    vals = np.concatenate([np.asarray(v, dtype=np.float64) for v, _ in parts])
    idx = np.concatenate([np.asarray(i, dtype=np.int64) for _, i in parts])
    order = np.lexsort((idx, vals))[:k]
    return vals[order], idx[order]


KIND_EXIT, KIND_TRAIN, KIND_CHAINS, KIND_SCORE = 0, 1, 2, 3
ACQ_ORDER = ("EI", "LCB", "PI")
STATS_SCALARS = ("refits", "n_sum", "n_max", "refit_s", "propose_s", "prepare_s", "score_s", "polish_s")


def encode_histories(res):
    """{(trial, fold): history or None} -> f64 rows [t, f, n_vl, n_va, dropped_train,
    dropped_val, E, val_loss (E), val_acc (E)] (-1: absent)."""
    keys = sorted(res)
    E = 0
    for k in keys:
        h = res[k]
        if h is not None:
            extra = set(h) - {"val_loss", "val_acc", "dropped_train_samples", "dropped_val_samples"}
            if extra:
                raise TypeError(f"encode_histories: unsupported history keys {sorted(extra)}")
            E = max(E, len(h.get("val_loss", [])), len(h.get("val_acc", [])))
    rows = np.full((len(keys), 7 + 2 * E), np.nan)
    for r, (t, f) in enumerate(keys):
        h = res[(t, f)]
        rows[r, :7] = [t, f, -1, -1, -1, -1, E]
        if h is None:
            continue
        vl, va = list(h.get("val_loss", [])), list(h.get("val_acc", []))
        rows[r, 2], rows[r, 3] = len(vl), len(va)
        rows[r, 4] = h.get("dropped_train_samples", -1)
        rows[r, 5] = h.get("dropped_val_samples", -1)
        rows[r, 7:7 + len(vl)] = vl
        rows[r, 7 + E:7 + E + len(va)] = va
    return rows


def decode_histories(parts):
    out = {}
    for rows in parts:
        for row in rows:
            t, f, nvl, nva, dtr, dva, E = (int(v) for v in row[:7])
            if nvl < 0:
                out[(t, f)] = None
                continue
            h = {"val_loss": [float(v) for v in row[7:7 + nvl]], "val_acc": [float(v) for v in row[7 + E:7 + E + nva]]}
            if dtr >= 0:
                h["dropped_train_samples"] = dtr
            if dva >= 0:
                h["dropped_val_samples"] = dva
            out[(t, f)] = h
    return out


class DistributedEvaluator:
    """Shards work over torch.distributed ranks (one process per GPU); rank 0 drives.

    Every round is fixed-layout tensor collectives (``collectives.TensorChannel``:
    RCCL device tensors on ``nccl``, CPU tensors on gloo), announced by an int64
    header broadcast from rank 0 (the reference's tag-4 parameter sends and tag-2
    FOM receives, coordinator.py:140-150):
    * train -- the n x D suggestion table (values, type codes, trial ids)
      broadcast; (trial, fold) units LPT-sharded by FLOPs; per-unit history rows
      all-gathered;
    * chains -- the population's ask batches (``ChainJob.encode`` tables)
      broadcast, LPT-dealt by refit cost, each rank's batches (point tables),
      refit accounts and error text all-gathered;
    * score -- the fitted GP (observations, theta, y_opt, xi, kappa) broadcast,
      the candidates scattered M/W per rank, each rank's (value, index) top-k
      all-gathered and merged lowest-index-first (SURVEY §8e "EI"), used by
      :class:`ShardedScorer`.
    The only object broadcast is the optimizer configuration of the ask batches,
    once per search (and again only if it changes) -- never per round.
    """

    def __init__(self, local, group=None, chain_runner=None):
        import torch.distributed as dist

        from .collectives import TensorChannel

        self.local = local
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.ch = TensorChannel(dist, group)
        self.n_evaluated = 0
        self.chain_runner = chain_runner    # this rank's chains.ThreadChainExecutor (set by DistributedChainExecutor)
        self._job_config = None             # the ask batches' optimizer configuration (sent once)
        self.config_broadcasts = 0

    # ---- train ------------------------------------------------------------------
    def _train(self, n, d, has_ids, params_list=None, trial_ids=None):
        from .collectives import decode_points, encode_points

        table = None
        if self.rank == 0:
            vals, codes = encode_points(params_list) if n else (np.zeros((0, d)), np.zeros((0, d)))
            ids = np.asarray(trial_ids if has_ids else np.zeros(n), dtype=np.float64).reshape(n, 1)
            table = np.concatenate([vals.reshape(n, d), codes.reshape(n, d), ids], axis=1)
        t = self.ch.bcast(table, (n, 2 * d + 1))
        if self.rank != 0:
            params_list = decode_points(t[:, :d], t[:, d:2 * d])
            trial_ids = [int(v) for v in t[:, 2 * d]] if has_ids else None
        units = self.local.units(params_list)
        owner = lpt_assign([u[3] for u in units], self.world)
        mine = [u for u, o in zip(units, owner) if o == self.rank]
        if trial_ids is None:
            res = self.local.train_units(mine, seed_base=self.n_evaluated)
        else:
            res = self.local.train_units(mine, seed_base=self.n_evaluated, trial_ids=trial_ids)
        self.n_evaluated += len(params_list)
        parts = self.ch.gather_rows(encode_histories(res))
        return decode_histories(parts) if self.rank == 0 else None   # only rank 0 tells

    # ---- score ------------------------------------------------------------------
    def _score(self, m, d, n, k, mask, dm, fac=0, req=None):
        acqs = [a for i, a in enumerate(ACQ_ORDER) if mask >> i & 1]
        if fac:
            return self._score_factor(m, d, k, acqs, fac, req)
        head = None
        if self.rank == 0:
            head = [float(req.get("y_opt", 0.0)), float(req.get("xi", 0.01)), float(req.get("kappa", 1.96))]
            if dm:
                head += [float(req["amp"]), float(req["noise"])] + list(np.ravel(req["ls"]).astype(float)) + \
                    list(np.ravel(req["Xt"]).astype(float)) + list(np.ravel(req["y"]).astype(float))
        g = self.ch.bcast(head, (3 + (2 + dm + n * dm + n if dm else 0),))
        cand, s0, s1 = self.ch.scatter_rows(req["cand"] if self.rank == 0 else None, m, d)
        payload = {"y_opt": float(g[0]), "xi": float(g[1]), "kappa": float(g[2]), "acqs": acqs, "k": int(k),
                   "cand": cand}
        if dm:
            payload.update(amp=float(g[3]), noise=float(g[4]), ls=np.array(g[5:5 + dm]),
                           Xt=np.array(g[5 + dm:5 + dm + n * dm]).reshape(n, dm),
                           y=np.array(g[5 + dm + n * dm:5 + dm + n * dm + n]))
        part = local_topk(payload, 0, s1 - s0, device=self.local.device) if s1 > s0 else {}
        rows = np.full((len(acqs), 2 * k), np.nan)
        for r, a in enumerate(acqs):
            rows[r, k:] = -1.0
            if a in part:
                v, i = part[a]
                rows[r, :len(v)] = v
                rows[r, k:k + len(i)] = np.asarray(i, dtype=np.float64) + s0
        out = {}
        parts = self.ch.gather_rows(rows)
        for r, a in enumerate(acqs):
            lists = []
            for pr in parts:
                if len(pr):
                    idx = pr[r, k:].astype(np.int64)
                    keep = idx >= 0
                    lists.append((pr[r, :k][keep], idx[keep]))
            out[a] = merge_topk(lists, int(k))
        return out

    def _score_factor(self, m, d, k, acqs, wsb, req=None):
        """Sharded scoring of a fitted model: rank 0's prepared factor --
        the workspace ``mpo_gp_prepare`` wrote, ``DeviceGP.export_factor`` -- is
        broadcast as raw words, so no rank factorises again; the candidates are
        scattered, each rank scores its slice, the top-k rows are all-gathered."""
        import torch

        from .gp import DeviceGP

        dev = self.local.device if self.local.device is not None else torch.device("cuda", torch.cuda.current_device())
        lay_n = 4 + len(DeviceGP._PTRS)
        meta = layout = None
        if self.rank == 0:
            gp = req["est"].dev
            meta, layout, ws0 = gp.export_factor()
            meta = np.concatenate([meta, [float(req["y_opt"]), float(req.get("xi", 0.01)), float(req.get("kappa", 1.96))]])
        meta = self.ch.bcast(meta, (6,))
        layout = self.ch.bcast(layout, (lay_n,), dtype=np.int64)
        words = (wsb + 7) // 8
        # the workspace as int64 words: on RCCL straight between the GPUs' buffers
        if self.rank == 0 and self.ch.device.type == "cuda":
            buf = torch.zeros(words * 8, dtype=torch.uint8, device=self.ch.device)
            buf[:wsb].copy_(ws0[:wsb])
        elif self.rank == 0:
            buf = torch.zeros(words * 8, dtype=torch.uint8)
            buf[:wsb].copy_(ws0[:wsb].cpu())
        else:
            buf = torch.empty(words * 8, dtype=torch.uint8, device=self.ch.device)
        wv = buf.view(torch.int64)
        self.dist.broadcast(wv, src=0, group=self.group)
        if self.rank == 0:
            gp_local = gp
        else:
            ws = buf.to(dev) if buf.device != dev else buf
            gp_local = DeviceGP.from_factor(meta, layout, ws, device=dev)
        cand, s0, s1 = self.ch.scatter_rows(req["cand"] if self.rank == 0 else None, m, d, as_tensor=True)
        rows = np.full((len(acqs), 2 * k), np.nan)
        rows[:, k:] = -1.0
        if s1 > s0:
            top = _device_topk(types.SimpleNamespace(dev=gp_local), cand, float(meta[3]), tuple(acqs),
                               float(meta[4]), float(meta[5]), min(k, s1 - s0))
            for r, a in enumerate(acqs):
                v, i = top[a]
                rows[r, :len(v)] = v
                rows[r, k:k + len(i)] = np.asarray(i, dtype=np.float64) + s0
        out = {}
        parts = self.ch.gather_rows(rows)
        for r, a in enumerate(acqs):
            lists = []
            for pr in parts:
                if len(pr):
                    idx = pr[r, k:].astype(np.int64)
                    keep = idx >= 0
                    lists.append((pr[r, :k][keep], idx[keep]))
            out[a] = merge_topk(lists, int(k))
        return out

    # ---- chains -----------------------------------------------------------------
    def _chains(self, J, cfg_new, blob_len, jobs=None, enc=None):
        """Every rank runs its LPT share of the ask batches; all ranks get all batches."""
        from . import optimizer as O
        from .collectives import decode_points, encode_points

        if cfg_new:
            box = [jobs[0].config if self.rank == 0 else None]
            self.dist.broadcast_object_list(box, src=0, group=self.group)   # setup, once per search
            self._job_config = box[0]
            self.config_broadcasts += 1
        meta = blob = None
        if self.rank == 0:
            meta = np.stack([e[0] for e in enc]) if enc else np.zeros((0, O.ChainJob.META), dtype=np.int64)
            blob = np.concatenate([e[1] for e in enc]) if enc else np.zeros(0)
        meta = self.ch.bcast(meta, (J, O.ChainJob.META), dtype=np.int64)
        blob = self.ch.bcast(blob, (blob_len,))
        if self.rank != 0:
            jobs, o = [], 0
            for row in meta:
                ln = int(row[-1])
                jobs.append(O.ChainJob.decode(row, blob[o:o + ln], self._job_config))
                o += ln
        owner = lpt_assign([j.cost for j in jobs], self.world)
        mine = [i for i, o in enumerate(owner) if o == self.rank]
        if self.chain_runner is None:
            raise RuntimeError("DistributedEvaluator: no chain runner on this rank")
        if self.rank != 0:
            O.reset_stats()
        # a failure on one rank is gathered like a result and raised on every rank,
        # so no rank is left blocked in the all-gather
        try:
            res, err = (self.chain_runner.run_now([jobs[i] for i in mine]) if mine else []), ""
        except Exception as e:  # noqa: BLE001 -- re-raised below on every rank
            res, err = [], f"rank {self.rank}: {type(e).__name__}: {e}"
        # batches: rows [job index, n points, D, values, codes]
        enc = []
        for i, (X, trace) in zip(mine, res):
            if trace is not None:
                raise NotImplementedError("refit traces (parity tests) do not cross ranks")
            v, c = encode_points([list(x) for x in X])
            enc.append(np.concatenate([[i, v.shape[0], v.shape[1] if v.size else 0], v.ravel(), c.ravel()]))
        width = max([len(e) for e in enc], default=3)
        rows = np.zeros((len(enc), width))
        for r, e in enumerate(enc):
            rows[r, :len(e)] = e
        st = O.STATS
        srow = np.array([[*(float(st[k_]) for k_ in STATS_SCALARS), float(len(st["samples"])),
                          *np.ravel(np.asarray(st["samples"], dtype=np.float64))]]) if self.rank != 0 else \
            np.zeros((0, 0))
        merged = [None] * len(jobs)
        for part in self.ch.gather_rows(rows):
            if self.rank != 0:
                continue                     # only rank 0 hands the batches to the optimizer
            for row in part:
                i, npts, dd = int(row[0]), int(row[1]), int(row[2])
                v = row[3:3 + npts * dd].reshape(npts, dd)
                c = row[3 + npts * dd:3 + 2 * npts * dd].reshape(npts, dd)
                merged[i] = (decode_points(v, c), None)
        for r, part in enumerate(self.ch.gather_rows(srow)):
            if r == 0 or self.rank != 0 or not len(part):
                continue
            row = part[0]
            ns = int(row[len(STATS_SCALARS)])
            d_ = {k_: row[j] for j, k_ in enumerate(STATS_SCALARS)}
            for k_ in ("refits", "n_sum", "n_max"):
                d_[k_] = int(d_[k_])
            smp = row[len(STATS_SCALARS) + 1:len(STATS_SCALARS) + 1 + 2 * ns].reshape(ns, 2)
            d_["samples"] = [(int(a), float(b)) for a, b in smp]
            O.merge_stats(d_)
        errors = [e for e in self.ch.gather_text(err) if e]
        if errors:
            raise RuntimeError("ask batches failed: " + "; ".join(errors))
        return merged

    # ---- the round loop ------------------------------------------------------
    def _serve_one(self):
        h = self.ch.header()
        kind = h[0]
        if kind == KIND_EXIT:
            return False
        if kind == KIND_TRAIN:
            self._train(h[1], h[2], h[3])
        elif kind == KIND_CHAINS:
            self._chains(h[1], h[2], h[3])
        elif kind == KIND_SCORE:
            self._score(*h[1:8])
        else:
            raise ValueError(f"unknown round {kind}")
        return True

    accepts_trial_ids = True

    def evaluate(self, params_list, trial_ids=None):
        """Rank 0: evaluate a batch over all ranks."""
        params_list = [list(p) for p in params_list]
        ids = None if trial_ids is None else [int(i) for i in trial_ids]
        n, d = len(params_list), (len(params_list[0]) if params_list else 0)
        self.ch.header([KIND_TRAIN, n, d, int(ids is not None)])
        return self.local.foms(params_list, self._train(n, d, ids is not None, params_list, ids))

    def chains(self, jobs):
        """Rank 0: run ask batches (optimizer.ChainJob) over all ranks -> [(X, trace)]."""
        jobs = list(jobs)
        cfg_new = bool(jobs) and (self._job_config is None or jobs[0].config != self._job_config)
        for j in jobs[1:]:
            if j.config != jobs[0].config:
                raise ValueError("chains: the batches of one round must share one optimizer configuration")
        enc = [j.encode() for j in jobs]
        blob_len = int(sum(len(b) for _, b in enc))
        self.ch.header([KIND_CHAINS, len(jobs), int(cfg_new), blob_len])
        return self._chains(len(jobs), cfg_new, blob_len, jobs, enc)

    def score(self, req):
        """Rank 0: a sharded acquisition request -> {acq: (values, indices)} top-k."""
        acqs = list(req["acqs"])
        bad = [a for a in acqs if a not in ACQ_ORDER]
        if bad:
            raise ValueError(f"score: unknown acquisitions {bad}")
        mask = sum(1 << ACQ_ORDER.index(a) for a in acqs)
        cand = np.asarray(req["cand"], dtype=np.float64)
        m, d = cand.shape
        dm = int(np.asarray(req["Xt"]).shape[1]) if "Xt" in req else 0
        n = int(np.asarray(req["Xt"]).shape[0]) if "Xt" in req else 0
        # a fitted model (ShardedScorer): its prepared factor is broadcast; a bare
        # (Xt, y, theta) request: every rank factorises it (local_topk)
        fac = int(req["est"].dev.export_factor()[2].numel()) if req.get("est") is not None else 0
        self.ch.header([KIND_SCORE, m, d, n, int(req["k"]), mask, dm, fac])
        got = self._score(m, d, n, int(req["k"]), mask, dm, fac, req)
        return {a: got[a] for a in acqs}

    def serve(self):
        """Ranks > 0: serve rounds until rank 0 sends the exit header."""
        while self._serve_one():
            pass

    def shutdown(self):
        if self.rank == 0:
            self.ch.header([KIND_EXIT])


class ShardedScorer:
    """Optimizer acquisition scoring split over the ranks of a
    :class:`DistributedEvaluator` (the candidate batch M/W per GPU, then a global
    lowest-index top-k); plugs into ``Optimizer(scorer=...)``.  Not pickled.

    Sharding costs a broadcast of rank 0's prepared GP factor (the workspace
    ``mpo_gp_prepare`` filled -- no rank factorises again), a scatter of the
    candidates and an all-gather of the per-rank top-k rows; scoring costs ~1.3 ms
    per million candidates on one GPU.  Below ``min_shard`` candidates (skopt's
    ``n_points`` is 10 000) the request is scored on rank 0 alone, where the
    fitted model is already resident -- the split pays only for large batches."""

    def __init__(self, dist_eval, min_shard=1_000_000):
        self.dist_eval = dist_eval
        self.min_shard = int(min_shard)
        self.sharded_requests = 0
        self.local_requests = 0

    def __call__(self, est, X, y_opt, acqs, xi, kappa, k):
        if len(X) < self.min_shard or self.dist_eval.world == 1:
            self.local_requests += 1
            return {a: idx for a, (vals, idx) in _device_topk(est, X, y_opt, acqs, xi, kappa, k).items()}
        self.sharded_requests += 1
        req = {"est": est, "cand": np.ascontiguousarray(X, dtype=np.float64), "y_opt": float(y_opt),
               "acqs": list(acqs), "xi": float(xi), "kappa": float(kappa), "k": int(k)}
        return {a: idx for a, (vals, idx) in self.dist_eval.score(req).items()}
