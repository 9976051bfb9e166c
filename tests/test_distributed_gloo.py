"""DistributedEvaluator over a 2-rank gloo group (CPU): rank 0 broadcasts the
batch, ranks train their LPT shard, per-unit results are all-gathered; the FOMs
equal the single-process ones (independent of the world size)."""
import os
import socket

import torch.distributed as dist
import torch.multiprocessing as mp

from mpi_opt_amd.blocks import DistributedEvaluator, TrialEvaluator
from mpi_opt_amd.models import BuilderFromFunction, mnist_space
from mpi_opt_amd.models import test_mnist as mnist_model_fn


class CpuEval(TrialEvaluator):
    """Stands in for the GPU training: deterministic per-unit 'history'."""

    def train_units(self, units, seed_base=0):
        return {(t, f): {"val_loss": [spec.nb_filters / 100.0 + 0.01 * f + 1e-4 * seed_base], "val_acc": [0.0]}
                for (t, f, spec, _) in units}


BATCHES = [[[10, 2, 2, 50, 0.1], [50, 5, 3, 200, 0.2], [30, 3, 4, 100, 0.5]], [[12, 2, 3, 60, 0.0]]]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ev = DistributedEvaluator(CpuEval(BuilderFromFunction(mnist_model_fn, mnist_space()), None, None, n_fold=3))
    if rank == 0:
        out = [ev.evaluate(b) for b in BATCHES]
        ev.shutdown()
        q.put(out)
    else:
        ev.serve()
    dist.destroy_process_group()


def test_two_rank_gloo_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = CpuEval(BuilderFromFunction(mnist_model_fn, mnist_space()), None, None, n_fold=3)
    want = [ref.evaluate(b) for b in BATCHES]
    assert got == want
