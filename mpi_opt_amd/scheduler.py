"""Ask/tell scheduler of the search CLI (``python -m mpi_opt_amd.search``).

The reference drives its search with ``Coordinator`` (/root/reference/
coordinator.py:7-150).  A maintainer of the reference keeps that file and swaps
only ``skopt.Optimizer`` and the MPI communicator.  This
module is the build's OWN scheduler for its CLI.  It exposes the same
observable protocol as the reference loop, pinned event for event by
``tests/golden/coordinator_trace.json`` (generated from the reference itself):

* a batch of ``optimizer.ask(num_iterations)`` suggestions is cached and
  consumed from its end; any refit discards it (coordinator.py:46-50, 73);
* every pending result is told in ONE ``optimizer.tell(X, Y)``, the optimizer is
  checkpointed with pickle after it, and ``target_fom`` stops the loop
  (coordinator.py:52-55, 63-79);
* a free block is found by re-shuffling the block list (``random.shuffle``) and
  polling the busy ones' result requests (coordinator.py:105-138);
* a launch sends the parameters to every rank of the block (tag 4) and posts one
  ``irecv`` on the block master (tag 2) (coordinator.py:140-150);
* the end sends ``None`` to every rank and joins a barrier; trials still in
  flight are not told (coordinator.py:98-101).

Beyond the reference it keeps wall-clock accounts (``timings``): seconds spent
inside the optimizer (ask / tell, i.e. GP refits and acquisition) and inside
result polls (which, with :class:`~mpi_opt_amd.blocks.PopulationComm`, is where
the device population trains).
"""
from __future__ import annotations

import pickle
import random
import time
from dataclasses import dataclass, field

from .chains import LazyBatch, resolve
from .tag_lookup import tag_lookup

PARAMS_TAG = tag_lookup("params")
RESULT_TAG = tag_lookup("result")


def default_optimizer(dimensions, random_state, **kwargs):
    from .optimizer import Optimizer

    return Optimizer(dimensions=dimensions, random_state=random_state, **kwargs)


@dataclass
class _Launch:
    """One trial in flight on one block."""

    params: list
    request: object


@dataclass
class SearchState:
    """Everything the loop accumulates (also what ``Coordinator`` exposes)."""

    param_list: list = field(default_factory=list)   # told parameters, in order
    fom_list: list = field(default_factory=list)     # their figures of merit
    best_params: object = None
    best_fom: object = None
    unsent: list = field(default_factory=list)       # (params, fom) awaiting tell
    suggestions: list = field(default_factory=list)  # cached ask batch
    stop: bool = False


class AskTellScheduler:
    """Bayesian-optimisation loop over ``num_blocks`` blocks of a communicator.

    ``comm`` needs ``Get_size``, ``send(obj, dest, tag)``, ``irecv(source, tag)``
    (returning an object with ``test() -> (done, value)``) and ``Barrier`` --
    an mpi4py communicator or :class:`~mpi_opt_amd.blocks.PopulationComm`.
    """

    #: callable(dimensions, random_state) -> optimizer (tests inject stubs)
    optimizer_factory = staticmethod(default_optimizer)
    random_state = 13579            # coordinator.py:33

    def __init__(self, comm, num_blocks, dimensions, checkpoint="coordinator.pkl", target_fom=None,
                 verbose=False, optimizer_kwargs=None):
        self.comm = comm
        self.num_blocks = int(num_blocks)
        self.dimensions = dimensions
        self.checkpoint = checkpoint
        self.target_fom = target_fom
        self.verbose = verbose
        self.optimizer = type(self).optimizer_factory(dimensions, self.random_state, **(optimizer_kwargs or {}))
        self.state = SearchState()
        self.inflight = {}          # block -> _Launch
        self.timings = {"ask_s": 0.0, "tell_s": 0.0, "poll_s": 0.0, "asks": 0, "tells": 0}
        ranks = comm.Get_size() - 1
        self.block_size = ranks // self.num_blocks

    # -- reference-compatible views ------------------------------------------------
    param_list = property(lambda self: self.state.param_list)
    fom_list = property(lambda self: self.state.fom_list)
    best_params = property(lambda self: self.state.best_params)
    best_fom = property(lambda self: self.state.best_fom)

    def _log(self, *a):
        if self.verbose:
            print("[scheduler]", *a, flush=True)

    # -- checkpoint ------------------------------------------------------------------
    def save(self, fn=None):
        with open(fn or self.checkpoint, "wb") as fh:
            pickle.dump(self.optimizer, fh)

    def load(self, fn=None):
        with open(fn or self.checkpoint, "rb") as fh:
            self.optimizer = pickle.load(fh)

    # -- optimizer side ----------------------------------------------------------------
    def _suggest(self, batch):
        st = self.state
        if not st.suggestions:
            t0 = time.perf_counter()
            X = self.optimizer.ask(batch)
            # a lazy batch (optimizer with a chain executor) is popped as unresolved
            # points; a list is copied (the optimizer's ask cache holds it)
            st.suggestions = X.points() if isinstance(X, LazyBatch) else list(X)
            self.timings["ask_s"] += time.perf_counter() - t0
            self.timings["asks"] += 1
        return st.suggestions.pop()

    def _flush_results(self):
        st = self.state
        if not st.unsent:
            return
        xs = [p for p, _ in st.unsent]
        ys = [f for _, f in st.unsent]
        t0 = time.perf_counter()
        res = self.optimizer.tell(xs, ys)
        self.timings["tell_s"] += time.perf_counter() - t0
        self.timings["tells"] += 1
        st.best_params, st.best_fom = res.x, res.fun
        self._log(f"told {len(xs)} results; best {st.best_fom} at {st.best_params}")
        st.suggestions = []
        st.unsent = []
        self.save()
        if self.target_fom and res.fun < self.target_fom:
            self._log(f"target {self.target_fom} reached")
            st.stop = True

    # -- block side ----------------------------------------------------------------------
    def _ranks_of(self, block):
        first = (block - 1) * self.block_size + 1
        return range(first, first + self.block_size)

    def _collect(self, block):
        """True if ``block`` is free now (never used, or its trial just reported)."""
        launch = self.inflight.get(block)
        if launch is None:
            return True
        t0 = time.perf_counter()
        done, fom = launch.request.test()
        self.timings["poll_s"] += time.perf_counter() - t0
        if not done:
            return False
        del self.inflight[block]
        st = self.state
        params = resolve(launch.params)       # trained, so its batch has resolved
        st.param_list.append(params)
        st.fom_list.append(fom)
        st.unsent.append((params, fom))
        self._log(f"block {block} reported {fom} for {params}")
        return True

    def _free_block(self):
        order = list(range(1, self.num_blocks + 1))
        while True:
            self._flush_results()
            random.shuffle(order)
            hit = next((b for b in order if self._collect(b)), None)
            if hit is not None:
                return hit

    def _launch(self, block, params):
        for r in self._ranks_of(block):
            self.comm.send(params, dest=r, tag=PARAMS_TAG)
        req = self.comm.irecv(source=self._ranks_of(block)[0], tag=RESULT_TAG)
        self.inflight[block] = _Launch(params, req)
        self._log(f"launched block {block}: {params}")

    def run(self, num_iterations=1):
        for _ in range(num_iterations):
            block = self._free_block()
            if self.state.stop:
                break
            self._launch(block, self._suggest(num_iterations))
        for r in range(1, self.comm.Get_size()):
            self.comm.send(None, dest=r, tag=PARAMS_TAG)
        self.comm.Barrier()
        self._log(f"done; best {self.state.best_fom} at {self.state.best_params}")
        return self.state
