"""Concurrent constant-liar chains: the optimizer side of the north_star search.

The reference re-asks a whole ``cl_min`` batch after every told result
(``Coordinator.fit`` empties ``next_params``, /root/reference/coordinator.py:73;
``ask`` refills it with ``optimizer.ask(num_iterations)``, :46-50).  skopt's
``ask(n)`` works on a copy: ``opt = self.copy(random_state=self.rng.randint(...))``
then n x (``opt._ask()``, ``opt._tell(x, lie)``), one GP refit per lie.  At
``-n 129 --block-size 2 --num-iterations 256`` that is 257 refits per told trial,
~49 000 in the search -- sequential inside one batch, but **batches are
independent of each other**: a batch is a pure function of the asking
optimizer's state and the seed it draws (:class:`~mpi_opt_amd.optimizer.ChainJob`),
and the asking optimizer never sees the batch's lies.  The only thing the
protocol consumes from a batch is the point popped for the launch, which is
not told before the block that trains it reports.

So the scheduler keeps the reference's order of tells and asks exactly (every
told point, every RandomState draw of the asking optimizer, every popped
point is the same), but an ``ask`` only records its :class:`ChainJob` and
returns a :class:`LazyBatch`; the batches run concurrently, and a point is
waited for when the population that trains it is about to start
(:class:`~mpi_opt_amd.blocks.PopulationComm`):

* :class:`ThreadChainExecutor` -- worker threads on one GPU, each with its own
  HIP stream (a refit is ~100 latency-bound L-BFGS-B rounds of small kernels;
  several chains keep the GPU busy, and ctypes releases the GIL while a round
  waits on its stream);
* :class:`ProcessChainExecutor` -- spawned worker processes, each with a few
  worker threads (the chains' host-side L-BFGS-B -- scipy's ``setulb`` -- holds
  the GIL, ~70 us per round: one interpreter saturates at ~4 chains);
* :class:`DistributedChainExecutor` -- the batches of one population dealt over
  the torch.distributed ranks (LPT on the refit cost), each rank running its
  share on its own worker threads, results all-gathered to rank 0.
"""
from __future__ import annotations

import queue
import threading
import time


class LazyBatch:
    """The future result of one ``ask(n)`` batch.

    It behaves as the list skopt's ``ask(n)`` returns, as far as the reference's
    ``Coordinator`` uses one (coordinator.py:46-50): truthiness and ``len`` count
    the entries not yet popped, and ``pop(-1)`` removes the last one and returns
    it as a :class:`LazyPoint` without waiting for the batch.  skopt hands out its
    cached list itself, so the Coordinator's pops consume the optimizer's ask
    cache; popping this batch (the optimizer's cache entry) does the same.
    Iteration and indexing resolve the batch and see the remaining entries."""

    def __init__(self, executor, job):
        self.executor, self.job = executor, job
        self._X = None
        self._trace = None
        self._error = None
        self._done = threading.Event()
        self._left = list(range(job.n_points))   # entries not popped yet, in order
        self.seq = None             # submission number (executor bookkeeping)
        self.run_s = None           # seconds the batch ran on its worker

    def __len__(self):
        return len(self._left)

    def __bool__(self):
        return bool(self._left)

    def pop(self, index=-1):
        """Remove entry ``index`` of the remaining ones; a :class:`LazyPoint` (no wait)."""
        return LazyPoint(self, self._left.pop(index))

    def done(self):
        return self._done.is_set()

    def _set(self, X=None, trace=None, error=None):
        self._X, self._trace, self._error = X, trace, error
        self._done.set()

    def result(self):
        if not self._done.is_set():
            self.executor.wait(self)
        if self._error is not None:
            raise self._error
        return self._X

    def points(self):
        """One :class:`LazyPoint` per batch entry (what the scheduler pops from)."""
        return [LazyPoint(self, i) for i in range(self.job.n_points)]

    # list-like access resolves the batch
    def __iter__(self):
        X = self.result()
        return iter([X[i] for i in self._left])

    def __getitem__(self, i):
        return self.result()[self._left[i]]


class LazyPoint:
    """Entry ``index`` of a :class:`LazyBatch`: resolves on first use."""

    __slots__ = ("batch", "index")

    def __init__(self, batch, index):
        self.batch, self.index = batch, index

    def value(self):
        return self.batch.result()[self.index]

    def __iter__(self):
        return iter(self.value())

    def __len__(self):
        return len(self.value())

    def __getitem__(self, i):
        return self.value()[i]

    def __repr__(self):
        if self.batch.done():
            return repr(self.value())
        return f"<pending ask batch #{self.batch.seq} [{self.index}]>"


def resolve(p):
    """A plain parameter list from a point that may be lazy."""
    return list(p.value()) if isinstance(p, LazyPoint) else p


def resolve_all(points):
    """Resolve many points, letting their executors dispatch all outstanding batches at once."""
    return [resolve(p) for p in points]


class ThreadChainExecutor:
    """Runs batches on ``workers`` threads, each with its own stream on ``device``.

    Batches start as soon as they are submitted, in submission order."""

    def __init__(self, device=None, workers=4, start=True):
        self.device = device
        self.workers = int(workers)
        self._q = queue.Queue()
        self._threads = []
        self._seq = 0
        self.busy_s = 0.0           # summed worker seconds spent in chains
        self.wait_s = 0.0           # seconds callers blocked waiting for a batch
        self.durations = []         # (submission number, seconds) per finished batch
        self._lock = threading.Lock()
        if start:
            for w in range(self.workers):
                t = threading.Thread(target=self._worker, name=f"chain-{w}", daemon=True)
                t.start()
                self._threads.append(t)

    def _worker(self):
        import torch

        stream = None
        if self.device is not None and torch.cuda.is_available():
            dev = torch.device(self.device)
            torch.cuda.set_device(dev)
            stream = torch.cuda.Stream(dev)
        while True:
            batch = self._q.get()
            if batch is None:
                return
            t0 = time.perf_counter()
            try:
                if stream is not None:
                    with torch.cuda.stream(stream):
                        X, trace = batch.job.run(self.device)
                        stream.synchronize()
                else:
                    X, trace = batch.job.run(self.device)
                batch.run_s = time.perf_counter() - t0
                batch._set(X, trace)
            except BaseException as e:  # noqa: BLE001 -- re-raised by result()
                batch._set(error=e)
            with self._lock:
                self.busy_s += time.perf_counter() - t0
                self.durations.append((batch.seq, batch.run_s))

    def submit(self, job):
        b = LazyBatch(self, job)
        b.seq = self._seq
        self._seq += 1
        self._q.put(b)
        return b

    def run_now(self, jobs):
        """Run ``jobs`` on the workers and wait: [(X, trace)] in order (a rank's share)."""
        batches = [self.submit(j) for j in jobs]
        out = []
        for b in batches:
            X = b.result()
            out.append((X, b._trace))
        return out

    def wait(self, batch):
        t0 = time.perf_counter()
        batch._done.wait()
        self.wait_s += time.perf_counter() - t0

    def close(self):
        for _ in self._threads:
            self._q.put(None)
        for t in self._threads:
            t.join()
        self._threads = []


def _process_init(device):
    """Chain worker process: bind the GPU once (spawned interpreter, fresh HIP context)."""
    if device is not None:
        import torch

        torch.cuda.set_device(torch.device(device))


def _take_stats():
    """This process's refit accounts since the last call (then reset)."""
    from . import optimizer as O

    with O.STATS_LOCK:
        snap = {k: (list(v) if isinstance(v, list) else v) for k, v in O.STATS.items()}
    O.reset_stats()
    return snap


def _process_main(init, device, threads, in_q, out_q):
    """A chain worker process: ``threads`` chains at a time on its own
    :class:`ThreadChainExecutor`; results (and the refit accounts gathered since
    the previous result) go back in submission order."""
    import pickle

    init(device)
    local = ThreadChainExecutor(device, threads)
    pending = queue.Queue()

    def report():
        busy0 = 0.0
        while True:
            item = pending.get()
            if item is None:
                return
            seq, b = item
            b._done.wait()
            err = b._error
            if err is not None:
                try:
                    pickle.dumps(err)
                except Exception:  # noqa: BLE001 -- an unpicklable error travels as its repr
                    err = RuntimeError(repr(err))
            busy = local.busy_s
            out_q.put((seq, b._X, b._trace, err, _take_stats(), busy - busy0, b.run_s))
            busy0 = busy

    reporter = threading.Thread(target=report, daemon=True)
    reporter.start()
    while True:
        msg = in_q.get()
        if msg is None:
            break
        seq, job = msg
        pending.put((seq, local.submit(job)))
    pending.put(None)
    reporter.join()
    local.close()
    out_q.put(None)


class ProcessChainExecutor:
    """Runs batches in ``workers`` spawned processes sharing ``device``, each running
    ``threads`` batches at a time (its own HIP context and hardware queues, and its
    own interpreter: the chains' host side -- scipy's L-BFGS-B, which holds the GIL
    -- runs in parallel across processes).  Batches go to whichever process is free
    (one shared queue); their refit accounts are merged into this process's STATS."""

    def __init__(self, device=None, workers=2, threads=1):
        import multiprocessing as mp

        ctx = mp.get_context("spawn")
        self.device = None if device is None else str(device)
        self.workers, self.threads = int(workers), int(threads)
        self._in, self._out = ctx.Queue(), ctx.Queue()
        init = globals()["_process_init"]          # looked up now (tests substitute it)
        self._procs = [ctx.Process(target=_process_main, args=(init, self.device, self.threads, self._in, self._out),
                                   daemon=True) for _ in range(self.workers)]
        for pr in self._procs:
            pr.start()
        self._seq = 0
        self._batches = {}
        self._lock = threading.Lock()
        self.busy_s = 0.0
        self.wait_s = 0.0
        self.durations = []
        self._collector = threading.Thread(target=self._collect, daemon=True)
        self._collector.start()

    def _collect(self):
        from . import optimizer as O

        live = len(self._procs)
        while live:
            try:
                msg = self._out.get(timeout=1.0)
            except queue.Empty:
                dead = [pr for pr in self._procs if pr.exitcode not in (None, 0)]
                if dead:   # a worker died: fail every batch still outstanding
                    with self._lock:
                        outstanding, self._batches = list(self._batches.values()), {}
                    for b in outstanding:
                        b._set(error=RuntimeError(f"chain worker process exited with {dead[0].exitcode}"))
                    return
                continue
            if msg is None:
                live -= 1
                continue
            seq, X, trace, err, stats, busy, run_s = msg
            O.merge_stats(stats)
            with self._lock:
                self.busy_s += busy
                self.durations.append((seq, run_s))
                b = self._batches.pop(seq)
            b.run_s = run_s
            b._set(X, trace, err)

    def submit(self, job):
        b = LazyBatch(self, job)
        with self._lock:
            b.seq = self._seq
            self._seq += 1
            self._batches[b.seq] = b
        self._in.put((b.seq, job))
        return b

    def run_now(self, jobs):
        batches = [self.submit(j) for j in jobs]
        return [(b.result(), b._trace) for b in batches]

    def wait(self, batch):
        t0 = time.perf_counter()
        batch._done.wait()
        self.wait_s += time.perf_counter() - t0

    def close(self):
        for _ in self._procs:
            self._in.put(None)
        self._collector.join()
        for pr in self._procs:
            pr.join()


class DistributedChainExecutor:
    """Batches dealt over the ranks of a :class:`~mpi_opt_amd.blocks.DistributedEvaluator`.

    Rank 0 buffers submitted batches; the first wait dispatches every buffered
    batch in one ``("chains", jobs)`` round: LPT over the ranks by refit cost,
    each rank runs its share on its ``local`` :class:`ThreadChainExecutor`, and
    the batches (plus each rank's refit accounts) are all-gathered."""

    def __init__(self, dist_eval, local):
        self.dist_eval = dist_eval
        self.local = local
        self._pending = []
        self._seq = 0
        self.wait_s = 0.0
        self.rounds = 0
        dist_eval.chain_runner = local

    @property
    def busy_s(self):
        return self.local.busy_s

    def submit(self, job):
        b = LazyBatch(self, job)
        b.seq = self._seq
        self._seq += 1
        self._pending.append(b)
        return b

    def wait(self, batch):
        if batch.done():
            return
        t0 = time.perf_counter()
        pending, self._pending = self._pending, []
        if batch not in pending:
            raise RuntimeError("batch was never submitted to this executor")
        results = self.dist_eval.chains([b.job for b in pending])
        for b, (X, trace) in zip(pending, results):
            b._set(X, trace)
        self.rounds += 1
        self.wait_s += time.perf_counter() - t0

    def close(self):
        self.local.close()
