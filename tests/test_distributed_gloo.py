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


def _fake_local_topk(payload, s0, s1, device=None):
    """Stands in for the device scoring: deterministic per-candidate values with ties."""
    import numpy as np

    out = {}
    for j, acq in enumerate(payload["acqs"]):
        v = np.round(payload["cand"][s0:s1].sum(1) * 4) / 4 - j      # coarse: many ties
        order = np.lexsort((np.arange(s0, s1), v))[: min(payload["k"], s1 - s0)]
        out[acq] = (v[order], order + s0)
    return out


def _score_worker(rank, world, port, q):
    import numpy as np

    from mpi_opt_amd import blocks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blocks.local_topk = _fake_local_topk
    ev = DistributedEvaluator(CpuEval(BuilderFromFunction(mnist_model_fn, mnist_space()), None, None, n_fold=1))
    if rank == 0:
        cand = np.random.RandomState(0).uniform(size=(1001, 3))
        req = {"cand": cand, "acqs": ["EI", "LCB"], "k": 6}
        got = ev.score(req)
        ev.evaluate(BATCHES[1])       # a training round after a scoring round
        ev.shutdown()
        q.put((cand, {a: (v.tolist(), i.tolist()) for a, (v, i) in got.items()}))
    else:
        ev.serve()
    dist.destroy_process_group()


def test_sharded_scoring_merges_to_the_global_topk():
    """candidates split M/W per rank, per-rank (value, index) top-k
    all-gathered, merged lowest-index-first = the single-device top-k, ties too."""
    import numpy as np

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_score_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    cand, got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _fake_local_topk({"cand": cand, "acqs": ["EI", "LCB"], "k": 6}, 0, len(cand))
    for a in ("EI", "LCB"):
        assert got[a][1] == want[a][1].tolist() and got[a][0] == want[a][0].tolist()


def test_merge_topk_lexicographic():
    import numpy as np

    from mpi_opt_amd.blocks import merge_topk

    v, i = merge_topk([(np.array([0.5, 1.0]), np.array([7, 2])), (np.array([0.5, 0.25]), np.array([3, 9]))], 3)
    assert v.tolist() == [0.25, 0.5, 0.5] and i.tolist() == [9, 3, 7]


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


def _units_worker(rank, world, port, params, q):
    """Each rank: the LPT shard of the 256 x 5 (trial, fold) units it owns and its FLOPs."""
    from mpi_opt_amd.blocks import lpt_assign

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = CpuEval(BuilderFromFunction(mnist_model_fn, mnist_space()), None, None, n_fold=5)
    seen = []
    orig = local.train_units

    def record(units, seed_base=0):
        seen.extend((t, f, c) for (t, f, _, c) in units)
        return orig(units, seed_base)

    local.train_units = record
    ev = DistributedEvaluator(local)
    if rank == 0:
        foms = ev.evaluate(params)
        ev.shutdown()
    else:
        ev.serve()
        foms = None
    q.put((rank, foms, seen))
    dist.destroy_process_group()


def test_configs3_256_trials_x_5_folds_over_8_ranks():
    """BASELINE configs[3] sharding, rehearsed on 8 gloo ranks (CPU): 256 trials
    from option3's mnist space x 5 folds = 1 280 (trial, fold) units, LPT over
    the ranks by training FLOPs.  Every unit trains exactly once, the per-rank
    FLOPs are balanced within 10 % of the mean, and the FOMs equal one process
    evaluating the whole batch (unit seeds depend only on the unit)."""
    import numpy as np

    from mpi_opt_amd.space import Space

    space = Space(mnist_space())
    params = [list(p) for p in space.rvs(n_samples=256, random_state=np.random.RandomState(13579))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_units_worker, args=(r, 8, port, params, q)) for r in range(8)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(8)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    by_rank = {r: seen for r, _, seen in out}
    foms = next(f for r, f, _ in out if r == 0)
    units = sorted((t, f) for seen in by_rank.values() for (t, f, _) in seen)
    assert units == [(t, f) for t in range(256) for f in range(5)]
    loads = np.array([sum(c for (_, _, c) in by_rank[r]) for r in range(8)])
    assert loads.max() / loads.mean() <= 1.10, loads / loads.mean()
    ref = CpuEval(BuilderFromFunction(mnist_model_fn, mnist_space()), None, None, n_fold=5)
    assert foms == ref.evaluate(params)
