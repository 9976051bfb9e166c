"""DistributedEvaluator with the REAL device TrialEvaluator on the GPU box: two
ranks share cuda:0 over a gloo group (the node's 8-GPU launch is the driver's;
RCCL is the same code path with backend "nccl").  Rank 0 broadcasts each batch,
both ranks train their LPT shard of (trial, fold) units as device populations,
the histories are all-gathered -- and the FOMs are bit-identical to one process
training everything (unit seeds depend only on the unit; population isolation).
Reference: /root/reference/hyperparameter_search_option3.py:172-205,
coordinator.py:140-150."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

BATCHES = [[[10, 2, 2, 50, 0.1], [50, 5, 3, 200, 0.2], [30, 3, 4, 100, 0.5]], [[12, 2, 3, 60, 0.0], [40, 9, 2, 70, 0.3]]]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _evaluator():
    from mpi_opt_amd.blocks import TrialEvaluator
    from mpi_opt_amd.models import BuilderFromFunction, mnist_space
    from mpi_opt_amd.models import test_mnist as mnist_fn
    from mpi_opt_amd.population import synthetic_mnist

    x, y = synthetic_mnist(1000, seed=1, device="cuda:0")
    return TrialEvaluator(BuilderFromFunction(mnist_fn, mnist_space()), x, y, n_fold=2, epochs=1, device="cuda:0")


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from mpi_opt_amd.blocks import DistributedEvaluator

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ev = DistributedEvaluator(_evaluator())
    if rank == 0:
        out = [ev.evaluate(b) for b in BATCHES]
        ev.shutdown()
        q.put((out, ev.n_evaluated))
    else:
        ev.serve()
        q.put(("served", len(ev.local.units(BATCHES[0]))))
    dist.destroy_process_group()


def test_two_ranks_on_one_gpu_match_single_process():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dist_out = next(g for g in got if g[0] != "served")
    single = _evaluator()
    want = [single.evaluate(b) for b in BATCHES]
    assert dist_out[0] == want
    assert dist_out[1] == sum(len(b) for b in BATCHES)


TOLD = 12       # past n_initial_points = 10: the GP is fitted and the acquisition scored


def _told_points():
    import numpy as np

    rng = np.random.RandomState(4)
    X = [[int(rng.randint(10, 51)), int(rng.randint(2, 11)), int(rng.randint(2, 11)), int(rng.randint(50, 201)),
          float(rng.uniform())] for _ in range(TOLD)]
    y = [float(0.3 + 0.05 * np.sin(i)) for i in range(TOLD)]
    return X, y


def _opt(scorer=None):
    from mpi_opt_amd.models import mnist_space
    from mpi_opt_amd.optimizer import Optimizer

    return Optimizer(mnist_space(), random_state=13579, device="cuda:0", scorer=scorer,
                     acq_optimizer_kwargs={"n_points": 20000})


def _opt_worker(rank, world, port, q):
    import torch.distributed as dist

    from mpi_opt_amd.blocks import DistributedEvaluator, ShardedScorer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ev = DistributedEvaluator(_evaluator())
    if rank == 0:
        import pickle

        opt = _opt(ShardedScorer(ev, min_shard=0))      # force the split (default: >= 1M candidates only)
        X, y = _told_points()
        opt.tell(X, y)
        nxt = opt.ask()
        batch = opt.ask(3)
        # resume from a checkpoint (search --previous-result): the scorer is re-attached
        o2 = pickle.loads(pickle.dumps(opt))
        assert o2.scorer is None
        o2.set_runtime(device="cuda:0", scorer=opt.scorer)
        before = opt.scorer.sharded_requests
        o2.tell(list(batch[0]), 0.5)
        resumed = o2.ask()
        assert opt.scorer.sharded_requests > before
        ev.shutdown()
        q.put((list(nxt), [list(b) for b in batch], list(resumed)))
    else:
        ev.serve()
        q.put("served")
    dist.destroy_process_group()


def test_sharded_optimizer_scoring_matches_single_gpu():
    """The Optimizer's acquisition split over 2 ranks (ShardedScorer)
    proposes exactly the single-GPU points: same tell history, same next point,
    same cl_min batch."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_opt_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dist_out = next(g for g in got if g != "served")
    opt = _opt()
    X, y = _told_points()
    opt.tell(X, y)
    assert dist_out[0] == list(opt.ask())
    batch = opt.ask(3)
    assert dist_out[1] == [list(b) for b in batch]
    opt.tell(list(batch[0]), 0.5)
    assert dist_out[2] == list(opt.ask())


def _search_args(workers):
    from mpi_opt_amd import search

    return search.make_parser().parse_args(
        ["--world-size", "13", "--block-size", "2", "--n-fold", "2", "--num-iterations", "18", "--epochs", "1",
         "--n-samples", "1000", "--chain-workers", str(workers)])


def _search_worker(rank, world, port, tmp, q):
    import random

    import torch.distributed as dist

    from mpi_opt_amd import search

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    random.seed(11)
    args = _search_args(2)
    args.checkpoint = os.path.join(tmp, f"d{rank}.pkl")
    rep = search.run_search(args)
    if rank == 0:
        q.put({k: rep[k] for k in ("told_params", "told_foms", "trained_params", "populations")} |
              {"refits": rep["gp"]["refits"]})
    else:
        q.put("served")
    dist.destroy_process_group()


def test_search_with_chains_over_two_ranks_matches_one_process(tmp_path):
    """The search CLI's distributed path with the GP in the loop: 2 gloo ranks on
    cuda:0 train LPT shards of each population and run LPT shares of its cl_min
    ask batches (DistributedChainExecutor over 2 worker threads per rank); the told
    points, FOMs, trained trials and refit count equal one process asking inline."""
    import random

    import torch.multiprocessing as mp

    from mpi_opt_amd import optimizer as O
    from mpi_opt_amd import search

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_search_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=280) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dist_out = next(g for g in got if g != "served")
    random.seed(11)
    args = _search_args(0)
    args.checkpoint = str(tmp_path / "s.pkl")
    O.reset_stats()
    rep = search.run_search(args)
    assert dist_out["populations"] == rep["populations"] == [6, 6, 6]
    assert dist_out["told_params"] == rep["told_params"] and dist_out["told_foms"] == rep["told_foms"]
    assert dist_out["trained_params"] == rep["trained_params"]
    assert dist_out["refits"] == rep["gp"]["refits"]
