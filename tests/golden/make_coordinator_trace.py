"""Generate ``tests/golden/coordinator_trace.json`` from the REFERENCE
``/root/reference/coordinator.py`` (runs only in the build container; the
reference does not travel).  ``skopt`` is replaced by a deterministic stub and
MPI by a fake communicator, so the trace pins the Coordinator's scheduling
protocol exactly: ask caching + pop(-1) (coordinator.py:46-50), fit clearing the
cache (:63-79), shuffle + busy poll of blocks (:105-138), per-rank sends and
the irecv from the block master (:140-150), the exit broadcast (:98-101) and the
untold tail of in-flight trials.

    python tests/golden/make_coordinator_trace.py
"""
import json
import os
import random
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))


class StubOptimizer:
    """Deterministic stand-in for skopt.Optimizer (only ask/tell are used)."""

    def __init__(self, dimensions, random_state=None, log=None):
        self.log = log if log is not None else []
        self.n_ask = 0

    def ask(self, n):
        self.n_ask += 1
        pts = [[self.n_ask * 100 + i, 0.5 * i] for i in range(n)]
        self.log.append(["ask", n, pts])
        return [list(p) for p in pts]

    def tell(self, X, Y):
        self.log.append(["tell", [list(x) for x in X], list(Y)])

        class R:
            pass

        r = R()
        i = min(range(len(Y)), key=lambda j: Y[j])
        r.x, r.fun = list(X[i]), Y[i]
        return r


class FakeRequest:
    def __init__(self, comm, block, result, delay):
        self.comm, self.block, self.result, self.left = comm, block, result, delay

    def test(self):
        self.left -= 1
        done = self.left <= 0
        self.comm.log.append(["test", self.block, done])
        return (done, self.result if done else None)


class FakeComm:
    """size = 1 + num_blocks*block_size; block b's master is rank (b-1)*bs+1."""

    def __init__(self, num_blocks, block_size, log):
        self.nb, self.bs, self.log = num_blocks, block_size, log
        self.pending = {}

    def Get_size(self):
        return 1 + self.nb * self.bs

    def send(self, obj, dest, tag):
        self.log.append(["send", dest, tag, obj])

    def irecv(self, source, tag):
        block = (source - 1) // self.bs + 1
        params = None
        for e in reversed(self.log):
            if e[0] == "send" and e[1] == source:
                params = e[3]
                break
        result = float(sum(params)) / 1000.0
        delay = 1 + (block * 7 + len(self.log)) % 4
        self.log.append(["irecv", source, tag])
        return FakeRequest(self, block, result, delay)

    def Barrier(self):
        self.log.append(["barrier"])


CURRENT_LOG = []


def run_reference(num_blocks, block_size, num_iterations, seed):
    global CURRENT_LOG
    sys.path.insert(0, "/root/reference")
    log = CURRENT_LOG = []
    if "skopt" not in sys.modules:
        sk = types.ModuleType("skopt")
        sk.Optimizer = lambda dimensions, random_state=None: StubOptimizer(dimensions, random_state, CURRENT_LOG)
        sys.modules["skopt"] = sk
    import coordinator as ref_coordinator  # noqa: E402

    random.seed(seed)
    comm = FakeComm(num_blocks, block_size, log)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            import builtins
            real_print = builtins.print
            builtins.print = lambda *a, **k: None
            c = ref_coordinator.Coordinator(comm, num_blocks, [(0, 1), (0.0, 1.0)])
            c.save = lambda fn="coordinator.pkl": log.append(["save"])
            c.run(num_iterations=num_iterations)
        finally:
            builtins.print = real_print
            os.chdir(cwd)
    return {"num_blocks": num_blocks, "block_size": block_size, "num_iterations": num_iterations,
            "seed": seed, "events": log, "best_params": c.best_params, "best_fom": c.best_fom,
            "param_list": c.param_list, "fom_list": c.fom_list}


# -- the INTEGRATION.md §3 drop-in: reference Coordinator + lazy ask batches + PopulationComm --------

class StubJob:
    """A ChainJob stand-in: ``n_points`` deterministic points, computed when run."""

    def __init__(self, n_ask, n_points):
        self.n_ask, self.n_points = n_ask, n_points
        self.cost = float(n_points)

    def run(self, device=None, scorer=None):
        return [[self.n_ask * 100 + i, 0.5 * i] for i in range(self.n_points)], None


class DeferredExecutor:
    """A chain executor that runs nothing until a batch is waited for, then runs
    every submitted batch in submission order (as DistributedChainExecutor
    dispatches a population's buffered batches) and logs ("resolve", seqs):
    the trace shows exactly when the protocol waits for its asks."""

    def __init__(self, log):
        self.log, self._pending, self._seq = log, [], 0

    def submit(self, job):
        from mpi_opt_amd.chains import LazyBatch

        b = LazyBatch(self, job)
        b.seq = self._seq
        self._seq += 1
        self._pending.append(b)
        return b

    def wait(self, batch):
        pending, self._pending = self._pending, []
        self.log.append(["resolve", [b.seq for b in pending]])
        for b in pending:
            X, trace = b.job.run()
            b._set(X, trace)

    def close(self):
        pass


class LazyStubOptimizer:
    """StubOptimizer whose ``ask(n)`` returns a :class:`mpi_opt_amd.chains.LazyBatch`
    run by a chain executor, cached until the next tell (skopt's ask cache)."""

    def __init__(self, executor, log):
        self.executor, self.log = executor, log
        self.n_ask = 0
        self.cache = {}

    def ask(self, n):
        if n in self.cache:
            self.log.append(["ask_cached", n])
            return self.cache[n]
        self.n_ask += 1
        b = self.executor.submit(StubJob(self.n_ask, n))
        self.log.append(["ask", n, b.seq])
        self.cache = {n: b}
        return b

    def tell(self, X, Y):
        from mpi_opt_amd.chains import resolve

        X = [list(resolve(x)) for x in X]
        self.log.append(["tell", X, list(Y)])
        self.cache = {}

        class R:
            pass

        r = R()
        i = min(range(len(Y)), key=lambda j: Y[j])
        r.x, r.fun = list(X[i]), Y[i]
        return r


class SumEvaluator:
    """FOM = sum(params) / 1000 per trial (the FakeComm's rule)."""

    def evaluate(self, params_list):
        return [float(sum(p)) / 1000.0 for p in params_list]


def recording_population_comm(num_blocks, block_size, log):
    """A PopulationComm that logs the wire protocol; a sent point that is still an
    unresolved lazy point is logged as ("lazy", batch, index)."""
    from mpi_opt_amd.blocks import PopulationComm
    from mpi_opt_amd.chains import LazyPoint

    class Rec(PopulationComm):
        def send(self, obj, dest, tag):
            if isinstance(obj, LazyPoint):
                what = ["lazy", obj.batch.seq, obj.index, obj.batch.done()]
            else:
                what = obj if obj is None else list(obj)
            log.append(["send", dest, tag, what])
            return super().send(obj, dest, tag)

        def irecv(self, source, tag):
            log.append(["irecv", source, tag])
            req = super().irecv(source, tag)
            inner = req.test

            def test():
                done, val = inner()
                log.append(["test", req.block, done])
                return done, val

            req.test = test
            return req

        def evaluate_pending(self):
            n0 = len(self.trained_params)
            super().evaluate_pending()
            log.append(["population", [list(map(float, p)) for p in self.trained_params[n0:]]])

        def Barrier(self):
            log.append(["barrier"])
            return super().Barrier()

    return Rec(num_blocks, block_size, SumEvaluator())


def _plain(p):
    from mpi_opt_amd.chains import resolve

    return [float(v) for v in resolve(p)]


def run_reference_lazy(num_blocks, block_size, num_iterations, seed):
    """The reference Coordinator, unchanged, with a lazy-batch optimizer and PopulationComm."""
    global CURRENT_LOG
    sys.path.insert(0, "/root/reference")
    if "skopt" not in sys.modules:
        sk = types.ModuleType("skopt")
        sk.Optimizer = lambda dimensions, random_state=None: StubOptimizer(dimensions, random_state, CURRENT_LOG)
        sys.modules["skopt"] = sk
    import coordinator as ref_coordinator  # noqa: E402
    log = CURRENT_LOG = []
    random.seed(seed)
    comm = recording_population_comm(num_blocks, block_size, log)
    ex = DeferredExecutor(log)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            import builtins
            real_print = builtins.print
            builtins.print = lambda *a, **k: None
            c = ref_coordinator.Coordinator(comm, num_blocks, [(0, 1), (0.0, 1.0)])
            c.optimizer = LazyStubOptimizer(ex, log)
            c.save = lambda fn="coordinator.pkl": log.append(["save"])
            c.run(num_iterations=num_iterations)
        finally:
            builtins.print = real_print
            os.chdir(cwd)
            ex.close()
    return {"num_blocks": num_blocks, "block_size": block_size, "num_iterations": num_iterations,
            "seed": seed, "events": log, "best_params": _plain(c.best_params), "best_fom": c.best_fom,
            "param_list": [_plain(p) for p in c.param_list], "fom_list": c.fom_list,
            "batches": list(comm.batches), "tail": [[_plain(p), f] for p, f in comm.tail]}


if __name__ == "__main__":
    cases = [run_reference(4, 5, 10, 0), run_reference(2, 2, 7, 3), run_reference(3, 3, 12, 11)]
    path = os.path.join(HERE, "coordinator_trace.json")
    json.dump(cases, open(path, "w"), indent=0)
    for c in cases:
        n_tell = sum(1 for e in c["events"] if e[0] == "tell")
        print(path, "blocks", c["num_blocks"], "events", len(c["events"]), "fits", n_tell, "told", len(c["fom_list"]))
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    lazy = [run_reference_lazy(4, 5, 10, 0), run_reference_lazy(2, 2, 7, 3), run_reference_lazy(3, 3, 12, 11),
            run_reference_lazy(8, 2, 16, 5)]
    path = os.path.join(HERE, "coordinator_lazy_trace.json")
    json.dump(lazy, open(path, "w"), indent=0)
    for c in lazy:
        print(path, "blocks", c["num_blocks"], "events", len(c["events"]), "populations", c["batches"],
              "told", len(c["fom_list"]), "tail", len(c["tail"]))
