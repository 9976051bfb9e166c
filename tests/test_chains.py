"""Concurrent cl_min chains (mpi_opt_amd.chains): the search with lazy ask
batches -- run on worker threads, or dealt over gloo ranks -- tells, asks and
trains exactly what the sequential protocol does.

The GP refit needs the GPU, so here ``Optimizer._fit_and_propose`` is replaced
by a CPU surrogate that keeps what matters for the equivalence: it depends on
every told point, updates the gp_hedge gains and consumes a data-dependent
number of RandomState draws (skopt's ``rng.multinomial``).  The device chains
are checked against the sequential ones in tests/test_search_gpu.py."""
import os
import pickle
import socket
import types

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from mpi_opt_amd import optimizer as O
from mpi_opt_amd.blocks import DistributedEvaluator, PopulationComm, TrialEvaluator
from mpi_opt_amd.chains import DistributedChainExecutor, LazyBatch, LazyPoint, ThreadChainExecutor
from mpi_opt_amd.models import BuilderFromFunction, mnist_space
from mpi_opt_amd.models import test_mnist as mnist_model_fn
from mpi_opt_amd.scheduler import AskTellScheduler


def fake_fit_and_propose(self):
    Xt = self.space.transform(self.Xi)
    y = np.asarray(self.yi, dtype=float)
    w = np.linalg.lstsq(np.c_[Xt, np.ones(len(y))], y, rcond=None)[0]

    def mean(Z):
        return np.c_[Z, np.ones(len(Z))] @ w

    if hasattr(self, "next_xs_"):
        self.gains_ -= mean(np.vstack(self.next_xs_))
    X = self.space.rvs_transformed(n_samples=64, random_state=self.rng)
    best = Xt[int(np.argmin(y))]
    self.next_xs_ = [X[int(np.argmin(mean(X) + k * ((X - best) ** 2).sum(1)))] for k in range(3)]
    logits = self.gains_ - np.max(self.gains_)
    probs = np.exp(logits)
    probs /= probs.sum()
    pick = int(np.argmax(self.rng.multinomial(1, probs)))
    self._next_x = self.space.inverse_transform(self.next_xs_[pick].reshape(1, -1))[0]
    self.models.append(types.SimpleNamespace(_dev=None, w=w))
    O._record_refit(len(y), 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)


class InstantEval:
    """FOM = a deterministic function of the trial's parameters."""

    def evaluate(self, params):
        return [float((p[0] * 0.013 + p[1] * 0.07 + p[3] * 0.001 + p[4]) % 1.0) for p in params]


class SeededEval(TrialEvaluator):
    """A TrialEvaluator whose 'training' depends on each unit's seed (its trial
    identity), as the device trainer's initial weights and dropout masks do."""

    def __init__(self):
        super().__init__(BuilderFromFunction(mnist_model_fn, mnist_space()), None, None, n_fold=2)

    def _train_units(self, units, tid):
        return {(t, f): {"val_loss": [(self._uid(tid(t), f) % 9973) / 9973.0], "val_acc": [0.0]}
                for (t, f, _, _) in units}


def _search(tmp, executor=None, world=9, block=2, iters=24, chunks=1, evaluator=None):
    nb = (world - 1) // block
    comm = PopulationComm(nb, block, evaluator or InstantEval(), chunks=chunks)
    kw = {"chain_executor": executor} if executor is not None else {}
    O.reset_stats()
    sched = AskTellScheduler(comm, nb, mnist_space(), checkpoint=os.path.join(tmp, "c.pkl"), optimizer_kwargs=kw)
    st = sched.run(num_iterations=iters)
    return {"told": [list(map(float, p)) for p in st.param_list], "foms": list(st.fom_list),
            "trained": [list(map(float, p)) for p in comm.trained_params], "batches": list(comm.batches),
            "tail": [(list(map(float, p)), f) for p, f in comm.tail], "refits": O.STATS["refits"],
            "best": (list(map(float, st.best_params)), st.best_fom)}


@pytest.fixture
def fake_gp(monkeypatch):
    monkeypatch.setattr(O.Optimizer, "_fit_and_propose", fake_fit_and_propose)


def test_lazy_threaded_search_equals_sequential(fake_gp, tmp_path):
    import random

    random.seed(5)
    want = _search(str(tmp_path))
    ex = ThreadChainExecutor(device=None, workers=3)
    try:
        random.seed(5)
        got = _search(str(tmp_path), ex)
    finally:
        ex.close()
    assert want["batches"] == [4, 4, 4, 4, 4, 4]
    assert want["refits"] > 100
    assert got == want


def test_lazy_batch_pops_without_touching_the_ask_cache(fake_gp):
    opt = O.Optimizer(mnist_space(), random_state=3)
    for x, y in zip(opt.ask(12), np.linspace(0, 1, 12)):
        opt.tell(x, float(y))
    seq = opt.ask(6)
    opt2 = O.Optimizer(mnist_space(), random_state=3)
    ex = ThreadChainExecutor(device=None, workers=2)
    try:
        opt2.chain_executor = ex
        for x, y in zip(opt2.ask(12), np.linspace(0, 1, 12)):   # a lazy batch iterates resolved
            opt2.tell(x, float(y))
        lazy = opt2.ask(6)
        assert isinstance(lazy, LazyBatch)
        pts = lazy.points()
        last = pts.pop()
        assert isinstance(last, LazyPoint) and list(last) == list(seq[-1])
        assert opt2.ask(6) is lazy                               # cached until the next tell
        assert [list(p) for p in lazy] == [list(p) for p in seq]
        opt2.tell(last, 0.5)                                      # tell resolves a lazy point
        assert opt2.Xi[-1] == list(seq[-1])
    finally:
        ex.close()


def test_checkpoint_without_new_attributes_resumes(fake_gp):
    """an Optimizer pickled before ``trace`` existed must resume."""
    opt = O.Optimizer(mnist_space(), random_state=1)
    for x, y in zip(opt.ask(11), np.linspace(0, 1, 11)):
        opt.tell(x, float(y))
    d = dict(opt.__dict__)
    d.pop("trace")
    d.pop("chain_executor")
    old = O.Optimizer.__new__(O.Optimizer)
    old.__dict__.update(d)
    blob = pickle.dumps(old)
    back = pickle.loads(blob)
    assert back.trace is None and back.chain_executor is None
    back.ask(3)
    back.copy(random_state=4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Local:
    """DistributedEvaluator's local trainer: no training, FOMs from InstantEval."""

    device = None

    def units(self, params_list):
        return [(t, 0, None, 1.0) for t in range(len(params_list))]

    def train_units(self, units, seed_base=0, trial_ids=None):
        return {(t, 0): None for (t, _, _, _) in units}

    def foms(self, params_list, results):
        return InstantEval().evaluate(params_list)


def _dist_worker(rank, world, port, tmp, q):
    import random

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    O.Optimizer._fit_and_propose = fake_fit_and_propose
    # count the pickled object collectives: the rounds must be tensor collectives only
    # (the optimizer configuration is broadcast once per search)
    calls = {"object": 0}
    for name in ("broadcast_object_list", "all_gather_object", "gather_object", "scatter_object_list"):
        orig = getattr(dist, name)

        def counted(*a, _orig=orig, **k):
            calls["object"] += 1
            return _orig(*a, **k)

        setattr(dist, name, counted)
    ev = DistributedEvaluator(_Local())
    ex = DistributedChainExecutor(ev, ThreadChainExecutor(device=None, workers=2))
    if rank == 0:
        random.seed(5)
        nb = 4
        comm = PopulationComm(nb, 2, ev)
        O.reset_stats()
        sched = AskTellScheduler(comm, nb, mnist_space(), checkpoint=os.path.join(tmp, "d.pkl"),
                                 optimizer_kwargs={"chain_executor": ex})
        st = sched.run(num_iterations=24)
        ev.shutdown()
        q.put({"told": [list(map(float, p)) for p in st.param_list], "foms": list(st.fom_list),
               "trained": [list(map(float, p)) for p in comm.trained_params], "batches": list(comm.batches),
               "refits": O.STATS["refits"], "rounds": ex.rounds, "object_calls": calls["object"],
               "config_broadcasts": ev.config_broadcasts})
    else:
        ev.serve()
    ex.close()
    dist.destroy_process_group()


def test_chains_dealt_over_gloo_ranks_equal_sequential(fake_gp, tmp_path):
    import random

    random.seed(5)
    want = _search(str(tmp_path))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, 3, port, str(tmp_path), q)) for r in range(3)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rounds = got.pop("rounds")
    assert rounds == len(want["batches"])       # one dispatch of buffered batches per population
    # every round was tensor collectives: the one object broadcast is the search's
    # optimizer configuration, sent with the first batch round
    assert got.pop("config_broadcasts") == 1 and got.pop("object_calls") == 1
    for k in ("told", "foms", "trained", "batches", "refits"):
        assert got[k] == want[k], k


def test_chunked_populations_equal_whole_populations(fake_gp, tmp_path):
    """--population-chunks: a population trained in parts, each as soon as its own
    ask batches resolve, leaves the search unchanged (told points, FOMs, trained
    trials, refits); the timeline still has one entry per population."""
    import random

    random.seed(5)
    want = _search(str(tmp_path), world=17, iters=40)
    for chunks in (2, 3, 8):
        ex = ThreadChainExecutor(device=None, workers=3)
        try:
            random.seed(5)
            got = _search(str(tmp_path), ex, world=17, iters=40, chunks=chunks)
        finally:
            ex.close()
        assert got == want, chunks


def test_chunked_populations_keep_each_trials_seed(fake_gp, tmp_path):
    """a trial's seed (initial weights, dropout masks) is its
    population base plus its block-order position, so training a population in
    parts (reordered by ask-batch submission) gives every trial the same seed and
    the search the same FOMs as one whole population."""
    import random

    random.seed(5)
    want = _search(str(tmp_path), world=17, iters=40, evaluator=SeededEval())
    assert len(set(want["foms"])) == len(want["foms"])          # the FOMs really are seed-dependent
    for chunks in (2, 3):
        ex = ThreadChainExecutor(device=None, workers=3)
        try:
            random.seed(5)
            got = _search(str(tmp_path), ex, world=17, iters=40, chunks=chunks, evaluator=SeededEval())
        finally:
            ex.close()
        assert got == want, chunks


class _SlowJob:
    n_points, cost = 1, 1.0

    def __init__(self, fail=False):
        self.fail = fail

    def run(self, device=None, scorer=None):
        import time

        time.sleep(0.2)
        if self.fail:
            raise ValueError("boom")
        return [[1]], None


def test_cancel_fails_queued_batches_instead_of_running_them():
    """on the search's error path the queued batches fail at once
    (close() does not run them first); a batch already running finishes."""
    import time

    ex = ThreadChainExecutor(device=None, workers=1)
    bs = [ex.submit(_SlowJob()) for _ in range(4)]
    time.sleep(0.05)
    ex.cancel("search failed")
    t0 = time.perf_counter()
    ex.close()
    assert time.perf_counter() - t0 < 0.5
    assert bs[0].result() == [[1]]
    for b in bs[1:]:
        with pytest.raises(RuntimeError, match="search failed"):
            b.result()


def test_worker_setup_failure_fails_its_batches(monkeypatch):
    """a worker whose device / stream setup fails does not die
    silently: every batch it takes fails with the setup error."""
    import torch

    def bad_set_device(dev):
        raise RuntimeError("no such device")

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "set_device", bad_set_device)
    ex = ThreadChainExecutor(device="cuda:7", workers=2)
    try:
        b = ex.submit(_SlowJob())
        with pytest.raises(RuntimeError, match="no such device"):
            b.result()
    finally:
        ex.close()


class _FailingRunner:
    def __init__(self, rank):
        self.rank = rank

    def run_now(self, jobs):
        if self.rank == 1:
            raise ValueError("chain broke on rank 1")
        return [([[0]], None) for _ in jobs]


def _err_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ev = DistributedEvaluator(_Local(), chain_runner=_FailingRunner(rank))
    try:
        if rank == 0:
            base = O.Optimizer(mnist_space(), random_state=0)
            ev.chains([O.ChainJob(base, 100 + i, 1, "cl_min") for i in range(4)])
        else:
            ev.serve()
        q.put((rank, "no error"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


def test_a_chain_failure_on_one_rank_raises_on_every_rank():
    """a rank whose chains raise joins the all-gather with its error,
    so the others do not block in it; every rank raises."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_err_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert all("chain broke on rank 1" in m for m in got.values()), got
