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
        self._cancelled = None      # set by cancel(): queued batches fail with it instead of running
        if start:
            for w in range(self.workers):
                t = threading.Thread(target=self._worker, name=f"chain-{w}", daemon=True)
                t.start()
                self._threads.append(t)

    def _worker(self):
        import torch

        stream = None
        try:
            if self.device is not None and torch.cuda.is_available():
                dev = torch.device(self.device)
                torch.cuda.set_device(dev)
                stream = torch.cuda.Stream(dev)
        except BaseException as e:  # noqa: BLE001 -- every batch this worker takes fails with it
            setup_error = e
        else:
            setup_error = None
        while True:
            batch = self._q.get()
            if batch is None:
                return
            if setup_error is not None or self._cancelled is not None:
                batch._set(error=setup_error or self._cancelled)
                continue
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

    def cancel(self, reason="ask batches cancelled"):
        """Fail every batch not started yet (the search's error path: close() then
        does not run ~256 refits per queued batch before the error surfaces)."""
        self._cancelled = RuntimeError(reason)

    def close(self):
        for _ in self._threads:
            self._q.put(None)
        for t in self._threads:
            t.join()
        self._threads = []


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
