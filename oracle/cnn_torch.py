"""torch-CPU fp32 restatement of single-trial MNIST-CNN training -- the CPU
baseline of the training legs (BASELINE.md:45-52, SURVEY §8d "CPU baseline").

TEST INFRASTRUCTURE ONLY (like the rest of ``oracle/``): imported by ``tests/``
and by ``bench.py``'s ``cpu_baseline`` legs, never by the product.

The reference trains each trial with Keras/TF on the block's ranks
(process_block.py:71-96 -> mpi_learn, [ext]).  None of that is installed, so the
baseline is the same network and update written with torch's CPU kernels and
autograd, fp32 -- what a framework CPU path does per batch:

    Conv2D(F, k, valid) -> relu -> Conv2D(F, k) -> relu -> MaxPool(p)
    -> Dropout(rate) -> Flatten (NHWC order) -> Dense(dense) -> relu
    -> Dropout(rate) -> Dense(10) -> softmax -> Keras binary_crossentropy
    Adam (Keras form, lr_t = lr*sqrt(1-b2^t)/(1-b1^t))

(mpiLAPI.py:138-176; option3:60-61, 270-275).  Weights use the Keras shapes of
``oracle/cnn.py`` so the two restatements can be checked against each other
(``tests/test_oracle_cnn_torch.py``); ``mask_fn`` injects the shared dropout
counter hash for that check, and the timing mode uses torch's own Bernoulli.

:func:`time_trials` runs ``concurrent`` trials at once in separate processes,
each with ``cores // concurrent`` threads -- the ``-n 21 --block-size 5``
layout's 4 concurrent blocks on the host cores -- and reports per-trial seconds
per train step and per validation batch.
"""
from __future__ import annotations

import math
import time

import numpy as np

NUM_CLASSES = 10
IMG = 28
BCE_EPS = 1e-7


def glorot_params(F, k, p, dense, seed):
    """Keras glorot_uniform kernels / zero biases, Keras shapes (float32)."""
    H2 = IMG - 2 * (k - 1)
    K1 = (H2 // p) ** 2 * F
    shapes = [("w1", (k, k, 1, F)), ("b1", (F,)), ("w2", (k, k, F, F)), ("b2", (F,)),
              ("w3", (K1, dense)), ("b3", (dense,)), ("w4", (dense, NUM_CLASSES)), ("b4", (NUM_CLASSES,))]
    rng = np.random.RandomState(seed)
    out = {}
    for name, shape in shapes:
        if name.startswith("w"):
            if len(shape) == 4:
                fan_in, fan_out = shape[0] * shape[1] * shape[2], shape[0] * shape[1] * shape[3]
            else:
                fan_in, fan_out = shape
            lim = math.sqrt(6.0 / (fan_in + fan_out))
            out[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
        else:
            out[name] = np.zeros(shape, np.float32)
    return out


class TorchTrial:
    """One test_mnist trial trained with torch CPU kernels (fp32 by default)."""

    def __init__(self, F, k, p, dense, params, lr=1e-3, dropout=0.25, mask_fn=None, dtype=None,
                 beta1=0.9, beta2=0.999, eps=1e-8):
        import torch

        self.torch = torch
        self.dtype = dtype or torch.float32
        self.F, self.k, self.p, self.dense = F, k, p, dense
        self.lr, self.rate, self.mask_fn = lr, dropout, mask_fn
        self.b1, self.b2, self.eps = beta1, beta2, eps
        t = lambda a: torch.tensor(np.asarray(a), dtype=self.dtype)   # noqa: E731
        # Keras layouts kept as the parameters; conv kernels are viewed as OIHW
        self.P = {n: t(v).requires_grad_(True) for n, v in params.items()}
        self.m = {n: torch.zeros_like(v) for n, v in self.P.items()}
        self.v = {n: torch.zeros_like(v) for n, v in self.P.items()}
        self.t = 0

    def forward(self, x, y, step=0, train=True):
        torch = self.torch
        F_ = torch.nn.functional
        P = self.P
        B = x.shape[0]
        xt = x.reshape(B, 1, IMG, IMG)
        a1 = F_.relu(F_.conv2d(xt, P["w1"].permute(3, 2, 0, 1), P["b1"]))
        a2 = F_.relu(F_.conv2d(a1, P["w2"].permute(3, 2, 0, 1), P["b2"]))
        pool = F_.max_pool2d(a2, self.p, self.p)
        flat = pool.permute(0, 2, 3, 1).reshape(B, -1)             # NHWC flatten (Keras)
        keep = 1.0 - self.rate
        if train and self.rate > 0:
            flat = flat * self._mask(step, 0, flat) / keep
        h = F_.relu(flat @ P["w3"] + P["b3"])
        if train and self.rate > 0:
            h = h * self._mask(step, 1, h) / keep
        prob = torch.softmax(h @ P["w4"] + P["b4"], dim=1)
        onehot = F_.one_hot(y.long(), NUM_CLASSES).to(self.dtype)
        pc = prob.clamp(BCE_EPS, 1 - BCE_EPS)
        per_sample = -(onehot * torch.log(pc) + (1 - onehot) * torch.log(1 - pc)).mean(dim=1)
        return per_sample

    def _mask(self, step, layer, like):
        torch = self.torch
        if self.mask_fn is not None:
            m = self.mask_fn(step, layer, like.numel(), self.rate)
            return torch.tensor(np.asarray(m).reshape(like.shape), dtype=self.dtype)
        return (torch.rand(like.shape, dtype=self.dtype) >= self.rate).to(self.dtype)

    def train_step(self, x, y, step=0):
        torch = self.torch
        loss = self.forward(x, y, step=step, train=True).mean()
        grads = torch.autograd.grad(loss, list(self.P.values()))
        self.t += 1
        lr_t = self.lr * math.sqrt(1.0 - self.b2 ** self.t) / (1.0 - self.b1 ** self.t)
        with torch.no_grad():
            for (n, p), g in zip(self.P.items(), grads):
                self.m[n].mul_(self.b1).add_(g, alpha=1 - self.b1)
                self.v[n].mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
                p.sub_(lr_t * self.m[n] / (self.v[n].sqrt() + self.eps))
        return float(loss.detach())

    def eval_batch(self, x, y):
        with self.torch.no_grad():
            return float(self.forward(x, y, train=False).sum())


def _time_one(job):
    """Worker: time ``steps`` train steps and ``val`` validation batches of one trial."""
    import torch

    (F, k, p, dense, threads, steps, val, warmup, seed) = job
    torch.set_num_threads(threads)
    rng = np.random.RandomState(seed)
    x = torch.from_numpy(rng.uniform(size=(100, IMG * IMG)).astype(np.float32))
    y = torch.from_numpy(rng.randint(0, NUM_CLASSES, size=100))
    tr = TorchTrial(F, k, p, dense, glorot_params(F, k, p, dense, seed))
    for s in range(warmup):
        tr.train_step(x, y, s)
    t0 = time.perf_counter()
    for s in range(steps):
        tr.train_step(x, y, warmup + s)
    t1 = time.perf_counter()
    for _ in range(val):
        tr.eval_batch(x, y)
    t2 = time.perf_counter()
    return (t1 - t0) / steps, (t2 - t1) / max(val, 1)


def time_trials(trials, concurrent=4, cores=None, steps=4, val=2, warmup=1):
    """Per-trial (s per train step, s per validation batch) at batch 100, with
    ``concurrent`` trials running at once in spawned processes of
    ``cores // concurrent`` torch threads each.  ``trials`` = [(F, k, p, dense)]."""
    import multiprocessing as mp

    cores = int(cores or 1)
    threads = max(1, cores // concurrent)
    jobs = [(int(F), int(k), int(p), int(d), threads, steps, val, warmup, i)
            for i, (F, k, p, d) in enumerate(trials)]
    with mp.get_context("spawn").Pool(concurrent) as pool:
        return pool.map(_time_one, jobs, chunksize=1), threads
