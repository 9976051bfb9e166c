"""Time the DenseNet population step (BASELINE config 5 geometry) on one GPU:
train step and eval step ms, algorithmic TFLOP/s vs the FP32 MFMA peak."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)
from mpi_opt_amd.densenet import DenseNetArch, DenseNetPopulation, flops_per_sample_fwd, flops_per_sample_train, \
    synthetic_cifar  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--members", type=int, default=32)
ap.add_argument("--batch", type=int, default=100)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--no-eval", action="store_true", help="train steps only (the bench's PMC traffic passes)")
args = ap.parse_args()

x, y = synthetic_cifar(n=5000, seed=0)
pop = DenseNetPopulation(DenseNetArch(), [1e-3] * args.members, batch=args.batch)
order = torch.stack([torch.randperm(5000, device="cuda", dtype=torch.int64).to(torch.int32)
                     for _ in range(args.members)])
for s in range(2):
    pop.train_step(x, y, order, s * args.batch)
torch.cuda.synchronize()
t0 = time.time()
for s in range(args.steps):
    pop.train_step(x, y, order, (s % 40) * args.batch)
torch.cuda.synchronize()
tt = (time.time() - t0) / args.steps
if args.no_eval:
    print(f"members {args.members} batch {args.batch}: train {tt*1e3:.2f} ms", flush=True)
    sys.exit(0)
t0 = time.time()
for s in range(args.steps):
    pop.eval_step(x, y, order, (s % 40) * args.batch)
torch.cuda.synchronize()
te = (time.time() - t0) / args.steps
fl = flops_per_sample_train(pop.layers) * args.batch * args.members
fe = flops_per_sample_fwd(pop.layers) * args.batch * args.members
print(f"members {args.members} batch {args.batch}: train {tt*1e3:.2f} ms ({fl/tt/1e12:.1f} TF/s, "
      f"{fl/tt/157.3e12*100:.1f}% FP32 peak), eval {te*1e3:.2f} ms ({fe/te/1e12:.1f} TF/s), "
      f"loss {pop.loss[0].item():.4f}", flush=True)
