"""torch-CPU fp32 restatement of one DenseNet trial -- the CPU baseline of the
DenseNet leg (BASELINE configs[4]; BASELINE.md:45-52).

TEST INFRASTRUCTURE ONLY (like the rest of ``oracle/``).

The same network and update as ``oracle/densenet.py`` (densenet.py:12-196,
base_model.py:57-92: BN(axis=1) of NHWC = statistics per image row, ELU,
same-padded bias-free convs, concat, 1x1 transition + AvgPool2, GAP + Dense +
softmax, clipped categorical CE, l2(1e-4) on every tensor, Keras Adam) written
with torch's CPU kernels and autograd in fp32 -- what a framework CPU path does
per batch.  :func:`time_trials` times ``concurrent`` trials at once in spawned
processes of ``cores // concurrent`` threads, at batch 100.
"""
from __future__ import annotations

import math
import time

import numpy as np

from .densenet import BN_EPS, BN_MOMENTUM, CE_EPS, L2, arch_layers, he_uniform_init


class TorchDenseNet:
    def __init__(self, layers, params, state, lr=1e-3, dtype=None, beta1=0.9, beta2=0.999, eps=1e-8):
        import torch

        self.torch = torch
        self.dtype = dtype or torch.float32
        self.layers = layers
        self.P = {k: torch.tensor(np.asarray(v), dtype=self.dtype).requires_grad_(True) for k, v in params.items()}
        self.S = {k: torch.tensor(np.asarray(v), dtype=self.dtype) for k, v in state.items()}
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        self.m = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.t = 0

    def _conv(self, z, w):                    # z NCHW, w [ks, ks, cin, cout] (Keras)
        ks = w.shape[0]
        return self.torch.nn.functional.conv2d(z, w.permute(3, 2, 0, 1), padding=(ks - 1) // 2)

    def _bn_elu(self, i, z, train):
        """BatchNormalization(axis=1) of the NHWC tensor = per image row h: in NCHW
        the statistics run over (batch, channel, width) for every h."""
        torch = self.torch
        g, b = self.P[f"g{i}"], self.P[f"b{i}"]
        if train:
            mean = z.mean(dim=(0, 1, 3))
            var = ((z - mean[None, None, :, None]) ** 2).mean(dim=(0, 1, 3))
            with torch.no_grad():
                self.S[f"mm{i}"].mul_(BN_MOMENTUM).add_(mean.detach(), alpha=1 - BN_MOMENTUM)
                self.S[f"mv{i}"].mul_(BN_MOMENTUM).add_(var.detach(), alpha=1 - BN_MOMENTUM)
        else:
            mean, var = self.S[f"mm{i}"], self.S[f"mv{i}"]
        inv = torch.rsqrt(var + BN_EPS)
        y = (z - mean[None, None, :, None]) * (inv * g)[None, None, :, None] + b[None, None, :, None]
        return torch.nn.functional.elu(y)

    def forward(self, x, y, train=True):
        """x [B, H, W, C] float tensor, y [B] int tensor -> (mean CE + l2, logits)."""
        torch = self.torch
        P = self.P
        feats = None
        xin = x.permute(0, 3, 1, 2)
        for i, ly in enumerate(self.layers):
            k = ly["kind"]
            if k == "conv0":
                feats = [self._conv(xin, P[f"w{i}"])]
            elif k == "dense":
                feats.append(self._conv(self._bn_elu(i, torch.cat(feats, 1), train), P[f"w{i}"]))
            elif k == "trans":
                t = self._conv(self._bn_elu(i, torch.cat(feats, 1), train), P[f"w{i}"])
                feats = [torch.nn.functional.avg_pool2d(t, 2)]
            else:
                g = self._bn_elu(i, torch.cat(feats, 1), train).mean(dim=(2, 3))
                logits = g @ P["wd"] + P["bd"]
        p = torch.softmax(logits, dim=1)
        p = p / p.sum(dim=1, keepdim=True)
        pc = p.clamp(CE_EPS, 1 - CE_EPS)
        ce = -torch.log(pc[torch.arange(len(y)), y.long()])
        return ce, logits

    def train_step(self, x, y):
        torch = self.torch
        ce, _ = self.forward(x, y, train=True)
        loss = ce.mean() + L2 * sum((v * v).sum() for v in self.P.values())
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
            ce, logits = self.forward(x, y, train=False)
            return float(ce.sum()), int((logits.argmax(1) == y.long()).sum())


def _time_one(job):
    import torch

    threads, steps, val, warmup, seed, B = job
    torch.set_num_threads(threads)
    layers = arch_layers()
    p, s = he_uniform_init(layers, seed)
    net = TorchDenseNet(layers, p, s, lr=1e-3)
    rng = np.random.RandomState(seed)
    x = torch.from_numpy(rng.uniform(size=(B, 32, 32, 3)).astype(np.float32))
    y = torch.from_numpy(rng.randint(0, 10, size=B))
    for _ in range(warmup):
        net.train_step(x, y)
    t0 = time.perf_counter()
    for _ in range(steps):
        net.train_step(x, y)
    t1 = time.perf_counter()
    for _ in range(val):
        net.eval_batch(x, y)
    t2 = time.perf_counter()
    return (t1 - t0) / steps, (t2 - t1) / max(val, 1)


def time_trials(n_trials, concurrent=4, cores=None, steps=2, val=1, warmup=1, batch=100):
    """Per-trial (s per train step, s per validation batch) of the reference grid
    DenseNet (depth 10, 3 blocks, growth 12, nb_filter 16, 32x32x3) at ``batch``."""
    import multiprocessing as mp

    threads = max(1, int(cores or 1) // concurrent)
    jobs = [(threads, steps, val, warmup, i, batch) for i in range(n_trials)]
    with mp.get_context("spawn").Pool(concurrent) as pool:
        return pool.map(_time_one, jobs, chunksize=1), threads
