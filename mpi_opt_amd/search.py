"""Hyper-parameter search driver: the option3 CLI on the MI355X engine.

    python -m mpi_opt_amd.search --block-size 5 --example mnist --epochs 10 \\
        --num-iterations 10 [--n-fold 5] [--world-size 21]
    python -m torch.distributed.run --nproc-per-node 8 -m mpi_opt_amd.search ...

Same flags and defaults as /root/reference/hyperparameter_search_option3.py:54-96
(make_parser) with the same sanity check (:51-52) and block arithmetic
(:174-181: ``num_blocks, left_over = divmod(size - 1, block_size)``, exit on a
leftover).  ``--world-size`` plays the role of ``mpirun -n`` (the number of
ranks the reference would have): it fixes how many trials run concurrently
(``num_blocks``).  Every trial trains as population members on the GPU(s)
instead of on MPI blocks.

Training flags: ``--loss`` (binary_crossentropy | categorical_crossentropy) and
``--optimizer`` (adam | sgd) select the member's loss and update rule in the
kernels; ``--early-stopping`` / ``--target-metric`` stop members per fold
(mpi_opt_amd.stopping); another value is refused with exit status 2.  Flags
that configure mpi_learn's Downpour/EASGD exchange (--sync-every, --easgd,
--elastic-*, --n-master, --n-process, --worker-optimizer) are accepted and
recorded but have no effect: a trial is trained synchronously on one GPU
(single-trial semantics).  ``--preload-data`` / ``--cache-data``
concern mpi_learn's file loader; the data here is resident in HBM.
"""
from __future__ import annotations

import argparse
import os
import sys


def make_parser():
    p = argparse.ArgumentParser(description="Bayesian hyper-parameter search on MI355X")
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--batch", help="batch size", default=100, type=int)
    p.add_argument("--epochs", help="number of training epochs", default=10, type=int)
    p.add_argument("--optimizer", help="optimizer for master to use (adam | sgd)", default="adam")
    p.add_argument("--loss", help="loss function (binary_crossentropy | categorical_crossentropy)",
                   default="binary_crossentropy")
    p.add_argument("--sync-every", default=1, type=int, dest="sync_every",
                   help="how often to sync weights with master (no effect: synchronous single-GPU trials)")
    p.add_argument("--preload-data", default=0, type=int, dest="data_preload",
                   help="mpi_learn data preloading (no effect here: the data is resident on the GPU)")
    p.add_argument("--cache-data", default="", dest="caching_dir",
                   help="mpi_learn data cache dir (no effect here: the data is resident on the GPU)")
    p.add_argument("--early-stopping", default=None, dest="early_stopping",
                   help="patience for early stopping: N (val_loss) or METRIC,~<,N / METRIC,~>,N "
                        "(Keras EarlyStopping semantics restated from the flag's help; mpi_learn is "
                        "un-vendored, so parity unpinned)")
    p.add_argument("--target-metric", default=None, dest="target_metric",
                   help="stop a fold once METRIC,OP,VALUE holds (e.g. val_acc,>,0.97; restated from the "
                        "flag's help, parity unpinned)")
    p.add_argument("--easgd", action="store_true", help="mpi_learn EASGD exchange (no effect here: trials train synchronously on one GPU)")
    p.add_argument("--worker-optimizer", dest="worker_optimizer", default="sgd",
                   help="mpi_learn worker optimizer (no effect here: trials train synchronously on one GPU)")
    p.add_argument("--elastic-force", type=float, default=0.9, help="EASGD (no effect here: trials train synchronously on one GPU)")
    p.add_argument("--elastic-lr", type=float, default=1.0, dest="elastic_lr", help="EASGD (no effect here: trials train synchronously on one GPU)")
    p.add_argument("--elastic-momentum", type=float, default=0, dest="elastic_momentum", help="EASGD (no effect here: trials train synchronously on one GPU)")
    p.add_argument("--block-size", type=int, default=2, help="number of ranks per block (reference MPI layout)")
    p.add_argument("--n-fold", type=int, default=1, dest="n_fold")
    p.add_argument("--n-master", type=int, default=1, dest="n_master", help="mpi_learn masters per block (no effect here: trials train synchronously on one GPU)")
    p.add_argument("--n-process", type=int, default=1, dest="n_process",
                   help="mpi_learn processes per worker (no effect here: trials train synchronously on one GPU)")
    p.add_argument("--num-iterations", type=int, default=10)
    p.add_argument("--previous-result", default=None, dest="previous_state")
    p.add_argument("--target-objective", type=float, default=None, dest="target_objective")
    p.add_argument("--example", default="mnist", choices=["topclass", "mnist", "gan"])
    # MI355X build additions
    p.add_argument("--world-size", type=int, default=21,
                   help="rank count of the reference's `mpirun -n` (sets concurrent trials)")
    p.add_argument("--n-samples", type=int, default=60000, help="synthetic MNIST-shape samples")
    p.add_argument("--synthetic-labels", default="uniform", choices=["uniform", "learnable"],
                   dest="synthetic_labels",
                   help="labels of the synthetic data: uniform random (SURVEY §8d; a flat objective) or a "
                        "fixed random linear teacher on the pooled image (learnable; trials differ)")
    p.add_argument("--data-dir", default=None,
                   help="directory of *.h5 files with `features` / `labels` (option3's mnist data, "
                        "/bigdata/shared/mnist/*.h5); first 70%% of the files train, the rest validate")
    p.add_argument("--lr", type=float, default=1e-3, help="Adam learning rate (mpi_learn default)")
    p.add_argument("--history-dir", default=None, help="write per-trial history JSON here")
    p.add_argument("--checkpoint", default="coordinator.pkl")
    p.add_argument("--ei-candidates", type=int, default=10000,
                   help="acquisition candidates per ask (skopt n_points); split over the GPUs when distributed")
    p.add_argument("--chain-workers", type=int, default=8,
                   help="concurrent cl_min ask batches per GPU (worker threads, one HIP stream each; their "
                        "refit rounds share launches); 0 runs every ask inline, as the reference's "
                        "Coordinator does")
    p.add_argument("--population-chunks", type=int, default=1, dest="population_chunks",
                   help="train each population in this many parts, each as soon as its ask batches "
                        "resolve (overlaps the remaining batches with training; results unchanged)")
    return p


def check_sanity(args):
    assert args.block_size > 1, "Block size must be at least 2 (master + worker)"


def check_training_flags(args):
    """--loss / --optimizer / --early-stopping / --target-metric configure the
    trials' training (option3:60-61, 66-69 -> Algo and MPIKFoldManager); a value
    the population kernels do not implement is refused, never ignored.
    Returns the parsed stopping rule (or None)."""
    from . import _lib
    from .stopping import StopRule

    if args.loss not in _lib.LOSS_CODES:
        raise ValueError(f"--loss {args.loss!r}: the population kernels implement {sorted(_lib.LOSS_CODES)}")
    if args.optimizer not in _lib.OPT_CODES:
        raise ValueError(f"--optimizer {args.optimizer!r}: the population kernels implement {sorted(_lib.OPT_CODES)}")
    return StopRule.from_args(args.early_stopping, args.target_metric)


#: flags of mpi_learn's asynchronous multi-process training that have no counterpart
#: here (a trial trains synchronously on one GPU): (dest, default)
NO_EFFECT_FLAGS = (("sync_every", 1), ("data_preload", 0), ("caching_dir", ""), ("easgd", False),
                   ("worker_optimizer", "sgd"), ("elastic_force", 0.9), ("elastic_lr", 1.0),
                   ("elastic_momentum", 0), ("n_master", 1), ("n_process", 1))


def no_effect_notes(args):
    """One note per no-effect flag set away from its default (printed, not silent)."""
    return [f"note: --{dest.replace('_', '-')}={getattr(args, dest)!r} has no effect here "
            f"(mpi_learn's multi-process exchange is not reproduced; trials train synchronously on one GPU)"
            for dest, dflt in NO_EFFECT_FLAGS if getattr(args, dest, dflt) != dflt]


def block_layout(world_size, block_size):
    """option3:174-181: (num_blocks, left_over)."""
    return divmod(world_size - 1, block_size)


def run_search(args, x=None, y=None, log=print, progress=None, on_population=None):
    """Run the option3 search for parsed ``args``; returns a report dict (rank 0)
    or None (ranks > 0, which serve their shards until rank 0 is done).

    The report splits the wall time into the optimizer (ask = GP refits of the
    cl_min batch + acquisition, tell = the refit on told results) and the
    device training of the populations, and counts the trials trained."""
    import time

    import torch

    from .blocks import DistributedEvaluator, PopulationComm, ShardedScorer, TrialEvaluator
    from .chains import DistributedChainExecutor, ThreadChainExecutor
    from .models import BuilderFromFunction, mnist_space, test_mnist
    from .population import synthetic_mnist
    from .scheduler import AskTellScheduler

    num_blocks, left_over = block_layout(args.world_size, args.block_size)
    stopping = check_training_flags(args)
    for note in no_effect_notes(args):
        log(note)
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import torch.distributed as _dist

    # a group the caller set up is used even at world size 1 (the RCCL path under test)
    if ws > 1 or (_dist.is_available() and _dist.is_initialized()):
        dist = _dist
        if not dist.is_initialized():
            torch.cuda.set_device(local)
            dist.init_process_group("nccl")
        # a caller that set up the group (bench.py) also chose this rank's device
        local = torch.cuda.current_device()
    dev = torch.device("cuda", local)
    provider = BuilderFromFunction(model_fn=test_mnist, parameters=mnist_space())
    holdout = None
    if x is None and args.data_dir:
        from .h5 import load_xy, split_files

        import numpy as np

        train_list, val_list = split_files(args.data_dir)
        (xt, yt), (xv, yv) = load_xy(train_list), load_xy(val_list)
        holdout = len(yt)
        xh, yh = np.concatenate([xt, xv]), np.concatenate([yt, yv])
        x, y = torch.from_numpy(xh).to(dev), torch.from_numpy(yh).to(dev)
        log(f"data: {len(train_list)} train / {len(val_list)} validation files, {holdout} / "
            f"{len(yh) - holdout} samples")
    if x is None:
        x, y = synthetic_mnist(args.n_samples, seed=0, device=dev, labels=args.synthetic_labels)
    evaluator = TrialEvaluator(provider, x, y, n_fold=args.n_fold, epochs=args.epochs, batch=args.batch,
                               lr=args.lr, device=dev, history_dir=args.history_dir, holdout=holdout,
                               progress=progress if (dist is None or dist.get_rank() == 0) else None,
                               loss=args.loss, optimizer=args.optimizer, stopping=stopping)
    local_eval = evaluator
    chains = None
    if args.chain_workers > 0:
        chains = ThreadChainExecutor(dev, workers=args.chain_workers)
    if dist is not None:
        evaluator = DistributedEvaluator(evaluator)
        if chains is not None:
            chains = DistributedChainExecutor(evaluator, chains)
        if evaluator.rank != 0:
            try:
                evaluator.serve()
            finally:
                if chains is not None:
                    chains.close()
            return None
    comm = PopulationComm(num_blocks, args.block_size, evaluator, chunks=args.population_chunks)

    def _population_done(i, entry):
        from . import optimizer as _o

        log(f"population {i}: {entry[3]} trials; {entry[0]:.1f} s before it, {entry[1]:.1f} s waiting for ask "
            f"batches, {entry[2]:.1f} s training; {_o.STATS['refits']} refits so far")
        if on_population is not None:
            on_population(i, entry, dict(_o.STATS))

    comm.on_population = _population_done
    opt_kw = {"device": dev, "acq_optimizer_kwargs": {"n_points": args.ei_candidates}}
    if chains is not None:
        opt_kw["chain_executor"] = chains                 # ask batches run concurrently (mpi_opt_amd.chains)
    if dist is not None:
        opt_kw["scorer"] = ShardedScorer(evaluator)       # candidates split M/W over the GPUs
    sched = AskTellScheduler(comm, num_blocks, provider.parameters, checkpoint=args.checkpoint,
                             target_fom=args.target_objective, verbose=args.verbose, optimizer_kwargs=opt_kw)
    from . import optimizer as _opt_mod

    _opt_mod.reset_stats()
    if args.previous_state:
        sched.load(args.previous_state)
        # the pickle carries no device state: re-attach this run's device and scorer
        sched.optimizer.set_runtime(device=dev, scorer=opt_kw.get("scorer"), chain_executor=chains)
    t0 = time.perf_counter()
    try:
        state = sched.run(num_iterations=args.num_iterations)
        wall = time.perf_counter() - t0
    except BaseException:
        if chains is not None:      # do not run the queued batches before the error surfaces
            (getattr(chains, "local", None) or chains).cancel("search failed")
        raise
    finally:
        if dist is not None:
            evaluator.shutdown()
        if chains is not None:
            chains.close()
    tm = sched.timings
    chain_wait = chains.wait_s if chains is not None else 0.0
    report = {
        "wall_s": wall,
        "trials_trained": comm.trials_trained,
        "trials_told": len(state.fom_list),
        "populations": list(comm.batches),
        "trained_params": [list(p) for p in comm.trained_params],
        "told_params": [list(p) for p in state.param_list], "told_foms": list(state.fom_list),
        "num_blocks": num_blocks,
        # seconds the search loop spent on the optimizer: asks (inline batches, or just
        # recording a lazy one), tells, and waiting for lazy batches before a population trains
        "optimizer_s": tm["ask_s"] + tm["tell_s"] + chain_wait,
        "ask_s": tm["ask_s"], "tell_s": tm["tell_s"], "asks": tm["asks"], "tells": tm["tells"],
        "chain_wait_s": chain_wait, "chain_workers": args.chain_workers,
        "population_chunks": args.population_chunks,
        "chain_pool": f"{args.chain_workers} threads" if chains is not None else None,
        "chain_busy_s": chains.busy_s if chains is not None else 0.0,
        # seconds each ask batch ran on its worker, in submission order (one per ask)
        "chain_run_s": [d for _, d in sorted(getattr(chains, "durations", []) or
                                             getattr(getattr(chains, "local", None), "durations", []))],
        "train_s": local_eval.train_s,
        # headline on TOLD trials (the ones the optimizer saw); the in-flight tail the
        # exit barrier trains (coordinator.py:98-101 never tells it) is reported apart
        "trials_per_hour": 3600.0 * len(state.fom_list) / wall if wall > 0 else None,
        "trained_per_hour": 3600.0 * comm.trials_trained / wall if wall > 0 else None,
        "tail_trials": len(comm.tail),
        # per population: [between populations (tells, asks, launches), waiting for ask batches, training, trials]
        "timeline": [list(t) for t in comm.timeline],
        "best_fom": state.best_fom, "best_params": state.best_params,
        "gp": dict(_opt_mod.STATS),     # refits (tell + every cl_min lie), their n, refit / proposal seconds
    }
    log(f"search done: {report['trials_trained']} trials trained ({report['trials_told']} told) in "
        f"{wall:.1f} s; optimizer {report['optimizer_s']:.2f} s, training {report['train_s']:.1f} s; "
        f"best {state.best_fom} at {state.best_params}")
    return report


def main(argv=None):
    args = make_parser().parse_args(argv)
    check_sanity(args)
    try:
        check_training_flags(args)
    except ValueError as e:
        print(f"error: {e}", file=sys.stderr)
        return 2
    if args.example != "mnist":
        print(f"example {args.example!r}: its data ({'LCD jets' if args.example == 'topclass' else '3D GAN'}) "
              "and model are outside the MNIST population engine", file=sys.stderr)
        return 2
    num_blocks, left_over = block_layout(args.world_size, args.block_size)
    if left_over:
        print("The last block is going to be made of {} nodes, make inconsistent block size {}".format(
            left_over, args.block_size))
        return 1
    run_search(args)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
