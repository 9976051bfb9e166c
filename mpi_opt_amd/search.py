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
instead of on MPI blocks; flags that configure mpi_learn's Downpour/EASGD
exchange (--sync-every, --easgd, --elastic-*, --n-master, --n-process,
--worker-optimizer) are accepted and recorded but have no effect: a trial is
trained synchronously on one GPU (single-trial semantics).
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
    p.add_argument("--optimizer", help="optimizer for master to use", default="adam")
    p.add_argument("--loss", help="loss function", default="binary_crossentropy")
    p.add_argument("--sync-every", default=1, type=int, dest="sync_every",
                   help="how often to sync weights with master (no effect: synchronous single-GPU trials)")
    p.add_argument("--preload-data", default=0, type=int, dest="data_preload")
    p.add_argument("--cache-data", default="", dest="caching_dir")
    p.add_argument("--early-stopping", default=None, dest="early_stopping")
    p.add_argument("--target-metric", default=None, dest="target_metric")
    p.add_argument("--easgd", action="store_true")
    p.add_argument("--worker-optimizer", dest="worker_optimizer", default="sgd")
    p.add_argument("--elastic-force", type=float, default=0.9)
    p.add_argument("--elastic-lr", type=float, default=1.0, dest="elastic_lr")
    p.add_argument("--elastic-momentum", type=float, default=0, dest="elastic_momentum")
    p.add_argument("--block-size", type=int, default=2, help="number of ranks per block (reference MPI layout)")
    p.add_argument("--n-fold", type=int, default=1, dest="n_fold")
    p.add_argument("--n-master", type=int, default=1, dest="n_master")
    p.add_argument("--n-process", type=int, default=1, dest="n_process")
    p.add_argument("--num-iterations", type=int, default=10)
    p.add_argument("--previous-result", default=None, dest="previous_state")
    p.add_argument("--target-objective", type=float, default=None, dest="target_objective")
    p.add_argument("--example", default="mnist", choices=["topclass", "mnist", "gan"])
    # MI355X build additions
    p.add_argument("--world-size", type=int, default=21,
                   help="rank count of the reference's `mpirun -n` (sets concurrent trials)")
    p.add_argument("--n-samples", type=int, default=60000, help="synthetic MNIST-shape samples")
    p.add_argument("--lr", type=float, default=1e-3, help="Adam learning rate (mpi_learn default)")
    p.add_argument("--history-dir", default=None, help="write per-trial history JSON here")
    p.add_argument("--checkpoint", default="coordinator.pkl")
    return p


def check_sanity(args):
    assert args.block_size > 1, "Block size must be at least 2 (master + worker)"


def block_layout(world_size, block_size):
    """option3:174-181: (num_blocks, left_over)."""
    return divmod(world_size - 1, block_size)


def main(argv=None):
    args = make_parser().parse_args(argv)
    check_sanity(args)
    if args.example != "mnist":
        print(f"example {args.example!r}: its data ({'LCD jets' if args.example == 'topclass' else '3D GAN'}) "
              "and model are outside the MNIST population engine", file=sys.stderr)
        return 2
    num_blocks, left_over = block_layout(args.world_size, args.block_size)
    if left_over:
        print("The last block is going to be made of {} nodes, make inconsistent block size {}".format(
            left_over, args.block_size))
        return 1

    import torch

    from .blocks import DistributedEvaluator, PopulationComm, TrialEvaluator
    from .coordinator import Coordinator
    from .models import BuilderFromFunction, mnist_space, test_mnist
    from .population import synthetic_mnist

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if ws > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    provider = BuilderFromFunction(model_fn=test_mnist, parameters=mnist_space())
    x, y = synthetic_mnist(args.n_samples, seed=0, device=dev)
    evaluator = TrialEvaluator(provider, x, y, n_fold=args.n_fold, epochs=args.epochs, batch=args.batch,
                               lr=args.lr, device=dev, history_dir=args.history_dir)
    if dist is not None:
        evaluator = DistributedEvaluator(evaluator)
        if evaluator.rank != 0:
            evaluator.serve()
            dist.destroy_process_group()
            return 0
    comm = PopulationComm(num_blocks, args.block_size, evaluator)
    Coordinator.checkpoint_file = args.checkpoint
    coord = Coordinator(comm, num_blocks, provider.parameters)
    if args.previous_state:
        coord.load(args.previous_state)
    if args.target_objective:
        coord.target_fom = args.target_objective
    coord.run(num_iterations=args.num_iterations)
    if dist is not None:
        evaluator.shutdown()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
