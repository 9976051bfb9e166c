"""Bayesian-optimisation coordinator: drop-in for /root/reference/coordinator.py.

Same constructor ``Coordinator(comm, num_blocks, opt_params)``, methods and
message protocol as the reference (coordinator.py:7-150), reproduced exactly --
pinned by tests/golden/coordinator_trace.json, generated from the reference
itself:

* ``ask(n)`` caches ``optimizer.ask(n)`` and pops from the end (:46-50);
* ``fit()`` tells every pending result in one batch, records the best point,
  clears the cached batch and checkpoints the optimizer with pickle (:63-79);
* ``run()`` waits for an idle block (fit, shuffle, poll every block) and sends
  the next parameters to every rank of it, then an ``irecv`` from the block
  master (:87-150); at the end it signals every rank with ``None`` and joins a
  barrier, leaving the last in-flight trials untold, as the reference does.

Only the optimizer and the communicator change: ``skopt.Optimizer`` becomes
:class:`mpi_opt_amd.optimizer.Optimizer` (device acquisition), and ``comm`` is
either an MPI communicator or a :class:`mpi_opt_amd.blocks.PopulationComm`,
which trains every launched block as members of one GPU population.
"""
from __future__ import annotations

import pickle
import random

from .tag_lookup import tag_lookup


def _default_optimizer(dimensions, random_state):
    from .optimizer import Optimizer

    return Optimizer(dimensions=dimensions, random_state=random_state)


class Coordinator(object):
    #: callable(dimensions, random_state) -> optimizer; replaced in tests
    optimizer_factory = staticmethod(_default_optimizer)
    checkpoint_file = "coordinator.pkl"

    def __init__(self, comm, num_blocks, opt_params):
        print("Coordinator initializing")
        self.comm = comm
        self.num_blocks = num_blocks
        self.opt_params = opt_params
        self.optimizer = type(self).optimizer_factory(self.opt_params, 13579)
        self.param_list = []
        self.fom_list = []
        self.block_dict = {}
        self.req_dict = {}
        self.best_params = None
        self.best_fom = None
        self.next_params = []
        self.to_tell = []
        self.ends_cycle = False
        self.target_fom = None

    def ask(self, n_iter):
        if not self.next_params:
            self.next_params = self.optimizer.ask(n_iter)
        return self.next_params.pop(-1)

    def save(self, fn=None):
        with open(fn or self.checkpoint_file, "wb") as d:
            pickle.dump(self.optimizer, d)

    def load(self, fn=None):
        fn = fn or self.checkpoint_file
        print("loading the coordinator optimizer from", fn)
        with open(fn, "rb") as d:
            self.optimizer = pickle.load(d)

    def fit(self):
        X = [o[0] for o in self.to_tell]
        Y = [o[1] for o in self.to_tell]
        if X and Y:
            print("Fitting from {} values".format(len(X)))
            res = self.optimizer.tell(X, Y)
            self.best_params = res.x
            self.best_fom = res.fun
            print("New best param estimate, with telling {} points : {}, with value {}".format(
                len(X), self.best_params, self.best_fom))
            self.next_params = []
            self.to_tell = []
            self.save()
            if self.target_fom and res.fun < self.target_fom:
                print("the optimization has reached the desired value at optimum", self.target_fom)
                self.ends_cycle = True

    def tell(self, params, result):
        self.to_tell.append((params, result))

    def run(self, num_iterations=1):
        for step in range(num_iterations):
            print("Coordinator iteration {}".format(step))
            next_block = self.wait_for_idle_block()
            if self.ends_cycle:
                print("Coordinator is skiping the iteration cycle")
                break
            next_params = self.ask(num_iterations)
            print("Next block: {}, next params {}".format(next_block, next_params))
            self.run_block(next_block, next_params)
        for proc in range(1, self.comm.Get_size()):
            self.comm.send(None, dest=proc, tag=tag_lookup("params"))
        self.comm.Barrier()
        print("Finished all iterations!")
        print("Best parameters found: {} with value {}".format(self.best_params, self.best_fom))

    def wait_for_idle_block(self):
        blocklist = list(range(1, self.num_blocks + 1))
        while True:
            self.fit()
            random.shuffle(blocklist)
            for cur_block in blocklist:
                if self.check_block(cur_block):
                    print("From coordinator, block {} is found idling, and can be used next".format(cur_block))
                    return cur_block

    def check_block(self, block_num):
        if block_num not in self.block_dict:
            return True
        done, result = self.req_dict[block_num].test()
        if not done:
            return False
        params = self.block_dict.pop(block_num)
        self.param_list.append(params)
        self.fom_list.append(result)
        print("Telling {} at {}".format(result, params))
        self.tell(params, result)
        del self.req_dict[block_num]
        return True

    def run_block(self, block_num, params):
        self.block_dict[block_num] = params
        block_size = int((self.comm.Get_size() - 1) / self.num_blocks)
        start = (block_num - 1) * block_size + 1
        end = block_num * block_size
        print("Launching block {}. Sending params to nodes from {} to {}".format(block_num, start, end))
        for proc in range(start, end + 1):
            self.comm.send(params, dest=proc, tag=tag_lookup("params"))
        self.req_dict[block_num] = self.comm.irecv(source=start, tag=tag_lookup("result"))
