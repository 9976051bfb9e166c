"""Device-resident DenseNet population (BASELINE config 5).

Replaces the per-block Keras training of ``DenseNet`` (/root/reference/densenet.py:135-196,
built by ``DenseNetModel.build`` base_model.py:61-72 / ``test_densenet`` mpiLAPI.py:197-201
and trained per MPI block by process_block.py:71-96).  The reference search grid
(base_model.py:84-92) fixes depth 10, 3 dense blocks, growth 12, nb_filter 16 and
dropout 0, and searches only the learning rate, so every member of a population
has the same architecture: each (trial, fold) member brings its own lr, weights,
BN moving statistics and sample order, and all of them step together through
``libmpo.so`` (csrc/densenet.hip).  torch only owns the device arenas.

Training semantics (as in the MNIST engine): one Keras ``Adam(lr)`` update per
batch on the batch gradient, ``categorical_crossentropy`` plus the l2(1e-4)
penalties of densenet.py, BN with batch statistics in training and moving
averages in evaluation; the figure of merit is the fold's validation loss
(mean CE + l2 penalty, as Keras reports ``val_loss``).
"""
from __future__ import annotations

import collections
import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr
from .population import kfold_split, train_folds  # noqa: F401 (kfold_split re-exported)

KIND_NAMES = {0: "conv0", 1: "dense", 2: "trans", 3: "head"}


@dataclass
class DenseNetArch:
    """``DenseNet(nb_classes, img_dim, depth, nb_dense_block, growth_rate, nb_filter)``
    (densenet.py:135); defaults are BASELINE config 5 (CIFAR-10 shape) with the
    base_model.py:84-92 grid values."""

    img_dim: tuple = (32, 32, 3)
    nb_classes: int = 10
    depth: int = 10
    nb_dense_block: int = 3
    growth_rate: int = 12
    nb_filter: int = 16

    def c_struct(self):
        H, W, C = self.img_dim
        return _lib.MpoDnArch(int(H), int(W), int(C), int(self.nb_classes), int(self.depth),
                              int(self.nb_dense_block), int(self.growth_rate), int(self.nb_filter))

    def layers(self):
        """Layer geometry (densenet.py:155-196), as the C plan builds it."""
        H, W, C0 = self.img_dim
        L = (self.depth - 4) // 3
        f, stage = self.nb_filter, 0
        out = [dict(kind="conv0", stage=0, H=H, W=W, cin=C0, cout=f, ks=3, coff=0)]
        for blk in range(self.nb_dense_block):
            for _ in range(L):
                out.append(dict(kind="dense", stage=stage, H=H, W=W, cin=f, cout=self.growth_rate, ks=3, coff=f))
                f += self.growth_rate
            if blk < self.nb_dense_block - 1:
                out.append(dict(kind="trans", stage=stage, H=H, W=W, cin=f, cout=f, ks=1, coff=0))
                H, W, stage = H // 2, W // 2, stage + 1
        out.append(dict(kind="head", stage=stage, H=H, W=W, cin=f, cout=self.nb_classes, ks=0, coff=0))
        return out

    def key(self):
        return (tuple(self.img_dim), self.nb_classes, self.depth, self.nb_dense_block, self.growth_rate,
                self.nb_filter)

    @classmethod
    def from_spec(cls, spec):
        """From a ``test_densenet`` / ``DenseNetModel`` JSON spec (models.py)."""
        return cls(img_dim=tuple(spec["img_dim"]), nb_classes=int(spec["nb_classes"]), depth=int(spec["depth"]),
                   nb_dense_block=int(spec["nb_dense_block"]), growth_rate=int(spec["growth_rate"]),
                   nb_filter=int(spec["nb_filter"]))


def param_shapes(layers):
    """Trainable tensors (Keras creation order) and BN moving-stat shapes."""
    P, S = {}, {}
    for i, ly in enumerate(layers):
        k = ly["kind"]
        if k == "conv0":
            P[f"w{i}"] = (3, 3, ly["cin"], ly["cout"])
            continue
        P[f"g{i}"] = (ly["H"],)
        P[f"b{i}"] = (ly["H"],)
        if k == "head":
            P["wd"] = (ly["cin"], ly["cout"])
            P["bd"] = (ly["cout"],)
        else:
            P[f"w{i}"] = (ly["ks"], ly["ks"], ly["cin"], ly["cout"])
        S[f"mm{i}"] = (ly["H"],)
        S[f"mv{i}"] = (ly["H"],)
    return P, S


def he_uniform_init(layers, seed):
    """Keras initialisers of densenet.py: he_uniform conv kernels (limit
    sqrt(6 / fan_in)), glorot-uniform dense kernel, zero bias, gamma 1, beta 0;
    moving mean 0 / variance 1 (float32)."""
    rng = np.random.RandomState(seed)
    P, S = param_shapes(layers)
    params = {}
    for n, shape in P.items():
        if n == "wd":
            lim = np.sqrt(6.0 / (shape[0] + shape[1]))
            params[n] = rng.uniform(-lim, lim, size=shape)
        elif n.startswith("w"):
            lim = np.sqrt(6.0 / (shape[0] * shape[1] * shape[2]))
            params[n] = rng.uniform(-lim, lim, size=shape)
        elif n.startswith("g"):
            params[n] = np.ones(shape)
        else:
            params[n] = np.zeros(shape)
    state = {n: (np.zeros(s) if n.startswith("mm") else np.ones(s)) for n, s in S.items()}
    return ({k: v.astype(np.float32) for k, v in params.items()},
            {k: v.astype(np.float32) for k, v in state.items()})


def flops_per_sample_fwd(layers):
    tot = 0
    for ly in layers:
        if ly["kind"] == "head":
            tot += 2 * ly["cin"] * ly["cout"]
        else:
            tot += 2 * ly["ks"] ** 2 * ly["cin"] * ly["cout"] * ly["H"] * ly["W"]
    return tot


def flops_per_sample_train(layers):
    """Forward + input gradient + weight gradient of every conv / dense layer,
    minus the initial conv's input gradient (not computed)."""
    c0 = layers[0]
    return 3 * flops_per_sample_fwd(layers) - 2 * 9 * c0["cin"] * c0["cout"] * c0["H"] * c0["W"]


def _pool_fused(H, W):
    """csrc/densenet.hip enqueue_forward: a transition's AvgPool2 runs in the 1x1
    conv's epilogue when the conv's row chunk (rows_per_chunk) is even."""
    return max(1, min(H, 128 // max(1, W))) % 2 == 0


def hbm_bytes_train(layers, batch, n_params):
    """Algorithmic HBM bytes of one train step of one member over ``batch``
    samples (f32), every tensor written once and read once per consuming kernel:
    forward -- each layer reads its input channels (BN + ELU folded into the
    consumer) and writes its output channels, the transition's AvgPool reads the
    conv output and writes the pooled stage (the conv writes the pooled stage itself
    when the pool is fused into its epilogue); backward -- each layer reads its
    output gradient and its input (for the weight gradient and the BN / ELU
    derivative), writes its input gradient (not for the initial conv), the pool
    reads / writes the gradient once; per member the parameters are read twice
    (forward, backward), the gradient written and read, Adam's m and v read and
    written and the parameters written (8 passes)."""
    per_sample = 0
    for ly in layers:
        hw = ly["H"] * ly["W"]
        if ly["kind"] == "head":
            per_sample += hw * ly["cin"] * 2 + hw * ly["cin"] * 2      # GAP read fwd; dGAP fold + input read bwd
            continue
        q = (ly["H"] // 2) * (ly["W"] // 2) * ly["cout"]
        if ly["kind"] == "trans" and (_pool_fused(ly["H"], ly["W"]) or _conv1x1_streamed(ly)):
            per_sample += hw * ly["cin"] + q                           # forward: conv + AvgPool2
            per_sample += hw * ly["cout"] + q                          # AvgPool2 backward
        else:
            per_sample += hw * (ly["cin"] + ly["cout"])                # forward
            if ly["kind"] == "trans":
                per_sample += 2 * (hw * ly["cout"] + q)                # AvgPool2 forward + backward
        per_sample += hw * (ly["cout"] + ly["cin"])                    # backward: dOut, input for wgrad / BN
        if ly["kind"] != "conv0":
            per_sample += hw * ly["cin"]                               # input gradient
    return 4 * (batch * per_sample + 8 * n_params)


def _conv1x1_streamed(ly):
    """csrc/densenet.hip conv1x1_ok for a transition: even H, W % 8 == 0, channels
    multiples of 4 and <= 64 (both its forward and its input gradient)."""
    H, W, cin, cout = ly["H"], ly["W"], ly["cin"], ly["cout"]
    return H % 2 == 0 and W % 8 == 0 and cin % 4 == 0 and cout % 4 == 0 and cin <= 64 and cout <= 64


def hbm_bytes_train_by_kernel(layers, batch, n_params):
    """Each DenseNet kernel family's own minimal HBM bytes for one train step of one
    member (f32; the kernels of csrc/densenet.hip as ``enqueue_forward`` /
    ``enqueue_backward`` launch them, every operand read once and every result
    written once per launch).  Unlike :func:`hbm_bytes_train` it counts the passes
    training-mode BatchNormalization needs by its data dependencies: the batch
    statistics of a site are read before any consumer can normalise (only the new
    growth channels -- totals carried over), and the backward's (sum dy, sum dy*xhat)
    reductions precede dx, so the reduce pass reads (dz, x) and the apply pass reads
    (dz, x[, dcat]) and writes dcat.  Weights, slabs and the per-row statistics are
    L2-sized and omitted; parameters as in :func:`hbm_bytes_train` (8 passes).
    Returns {family: bytes} (family = kernel name without template arguments)."""
    by = collections.defaultdict(float)
    prev = None
    for ly in layers:
        hw, cin, cout = ly["H"] * ly["W"], ly["cin"], ly["cout"]
        kind = ly["kind"]
        if kind == "conv0":
            by["dn_conv_kernel"] += hw * (cin + cout)                 # forward
            by["dn_wgrad3_kernel"] += hw * (cin + cout)               # backward: x, dOut
            prev = ly
            continue
        c0 = prev["cin"] if (prev is not None and prev["kind"] == "dense" and prev["stage"] == ly["stage"]
                             and prev["cin"] + prev["cout"] == cin) else 0
        by["dn_bn_stats_kernel"] += hw * (cin - c0)
        if kind == "head":
            by["dn_bn_apply_kernel"] += 2 * hw * cin                  # z stored for the GAP
            by["dn_head_fwd_kernel"] += hw * cin
            by["dn_bn_bwd_reduce_kernel"] += hw * cin                 # x (dz is the broadcast GAP gradient)
            by["dn_bn_bwd_apply_kernel"] += 2 * hw * cin              # x in, dcat out
            prev = ly
            continue
        if kind == "dense":
            by["dn_conv_kernel"] += hw * (cin + cout)                 # forward: cat in, growth slice out
            by["dn_wgrad3_kernel"] += hw * (cin + cout)
            by["dn_conv_kernel"] += hw * (cout + cin)                 # input gradient: dOut in, dz out
            by["dn_bn_bwd_reduce_kernel"] += 2 * hw * cin             # dz, x
            by["dn_bn_bwd_apply_kernel"] += 4 * hw * cin              # dz, x, dcat in; dcat out
        else:                                                         # transition
            q = (ly["H"] // 2) * (ly["W"] // 2) * cout
            # r05: the 1x1 convs stream on dn_conv1x1_kernel where it applies
            c1 = "dn_conv1x1_kernel" if _conv1x1_streamed(ly) else "dn_conv_kernel"
            if c1 == "dn_conv1x1_kernel" or _pool_fused(ly["H"], ly["W"]):
                by[c1] += hw * cin + q                                # AvgPool2 in the epilogue
            else:
                by[c1] += hw * (cin + cout)
                by["dn_pool_fwd_kernel"] += hw * cout + q
            by["dn_pool_bwd_kernel"] += q + hw * cout
            by["dn_wgrad1_kernel"] += hw * (cin + cout)
            by[c1] += hw * (cout + cin)
            by["dn_bn_bwd_reduce_kernel"] += 2 * hw * cin
            by["dn_bn_bwd_apply_kernel"] += 3 * hw * cin              # dz, x in; dcat stored
        prev = ly
    out = {k: 4.0 * batch * v for k, v in by.items()}
    out["dn_adam_kernel"] = 4.0 * 8 * n_params
    return out


class DenseNetPopulation:
    """``n`` same-architecture DenseNet members resident on one GPU."""

    def __init__(self, arch: DenseNetArch, lrs, batch=100, device=None, init=None, init_seed=0):
        self.arch = arch
        self.lrs = np.asarray(lrs, dtype=np.float32).reshape(-1)
        self.n = int(self.lrs.size)
        self.batch = int(batch)
        self.device = torch.device(device if device is not None else "cuda")
        L = lib()
        h = ctypes.c_void_p()
        a = arch.c_struct()
        check(L.mpo_dn_create(ctypes.byref(a), self.n, self.batch, ctypes.byref(h)), "mpo_dn_create")
        self._h = h
        sz = _lib.MpoDnSizes()
        check(L.mpo_dn_sizes(h, ctypes.byref(sz)), "mpo_dn_sizes")
        self.n_params, self.n_state = int(sz.n_params), int(sz.n_state)
        self.layers, self._offs = [], []
        geom = (ctypes.c_int32 * 8)()
        offs = (ctypes.c_int64 * 6)()
        for i in range(int(sz.n_layers)):
            check(L.mpo_dn_layer(h, i, geom, offs), "mpo_dn_layer")
            g = [int(v) for v in geom]
            self.layers.append(dict(kind=KIND_NAMES[g[0]], stage=g[1], H=g[2], W=g[3], cin=g[4], cout=g[5], ks=g[6],
                                    coff=g[7]))
            self._offs.append([int(v) for v in offs])
        self.param_shapes, self.state_shapes = param_shapes(self.layers)
        self._pslots, self._sslots = {}, {}
        for i, (ly, o) in enumerate(zip(self.layers, self._offs)):
            if ly["kind"] == "conv0":
                self._pslots[f"w{i}"] = o[0]
                continue
            self._pslots[f"g{i}"] = o[1]
            self._pslots[f"b{i}"] = o[2]
            if ly["kind"] == "head":
                self._pslots["wd"] = o[0]
                self._pslots["bd"] = o[5]
            else:
                self._pslots[f"w{i}"] = o[0]
            self._sslots[f"mm{i}"] = o[3]
            self._sslots[f"mv{i}"] = o[4]
        dev = self.device
        self.params = torch.zeros(self.n, self.n_params, dtype=torch.float32, device=dev)
        self.grads = torch.zeros_like(self.params)
        self.adam_m = torch.zeros_like(self.params)
        self.adam_v = torch.zeros_like(self.params)
        self.state = torch.zeros(self.n, self.n_state, dtype=torch.float32, device=dev)
        self.act = torch.zeros(int(sz.act_floats), dtype=torch.float32, device=dev)
        self.loss = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.val_loss_sum = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.val_correct = torch.zeros(self.n, dtype=torch.int32, device=dev)
        self._pen = torch.zeros(self.n, dtype=torch.float32, device=dev)
        lr_host = (ctypes.c_float * self.n)(*[float(v) for v in self.lrs])
        with torch.cuda.device(dev):
            check(L.mpo_dn_bind(h, ptr(self.params), ptr(self.grads), ptr(self.adam_m), ptr(self.adam_v),
                                ptr(self.state), ptr(self.act), ctypes.cast(lr_host, ctypes.c_void_p),
                                _lib.stream_handle(dev)), "mpo_dn_bind")
        if init is None:
            init = [he_uniform_init(self.layers, init_seed + i) for i in range(self.n)]
        for i, (p, s) in enumerate(init):
            self.set_params(i, p, s)
        self.step_count = 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().mpo_dn_destroy(h)
            except Exception:
                pass
            self._h = None

    # -- parameters ---------------------------------------------------------------
    def set_params(self, i, params, state=None):
        for n, shape in self.param_shapes.items():
            a = torch.from_numpy(np.asarray(params[n], dtype=np.float32).reshape(-1))
            off = self._pslots[n]
            self.params[i, off:off + a.numel()].copy_(a)
        if state is not None:
            for n, shape in self.state_shapes.items():
                a = torch.from_numpy(np.asarray(state[n], dtype=np.float32).reshape(-1))
                off = self._sslots[n]
                self.state[i, off:off + a.numel()].copy_(a)

    def get_params(self, i):
        host = self.params[i].cpu().numpy()
        return {n: host[self._pslots[n]:self._pslots[n] + int(np.prod(s))].reshape(s).copy()
                for n, s in self.param_shapes.items()}

    def get_grads(self, i):
        host = self.grads[i].cpu().numpy()
        return {n: host[self._pslots[n]:self._pslots[n] + int(np.prod(s))].reshape(s).copy()
                for n, s in self.param_shapes.items()}

    def get_state(self, i):
        host = self.state[i].cpu().numpy()
        return {n: host[self._sslots[n]:self._sslots[n] + int(np.prod(s))].reshape(s).copy()
                for n, s in self.state_shapes.items()}

    def reset_optimizer(self):
        self.adam_m.zero_()
        self.adam_v.zero_()
        self.step_count = 0

    # -- steps --------------------------------------------------------------------
    def train_step(self, x, labels, order, row0, step=None):
        """x [n,H,W,C] f32, labels [n] i32, order [n_members, L] i32 (device)."""
        step = self.step_count if step is None else int(step)
        with torch.cuda.device(self.device):
            check(lib().mpo_dn_train_step(self._h, ptr(x), ptr(labels), ptr(order), int(order.shape[1]), int(row0),
                                          step, ptr(self.loss), _lib.stream_handle(self.device)),
                  "mpo_dn_train_step")
        self.step_count = step + 1
        return self.loss

    def eval_reset(self):
        self.val_loss_sum.zero_()
        self.val_correct.zero_()

    def eval_step(self, x, labels, order, row0):
        with torch.cuda.device(self.device):
            check(lib().mpo_dn_eval_step(self._h, ptr(x), ptr(labels), ptr(order), int(order.shape[1]), int(row0),
                                         ptr(self.val_loss_sum), ptr(self.val_correct),
                                         _lib.stream_handle(self.device)), "mpo_dn_eval_step")

    def penalty(self):
        """Per-member l2 penalty 1e-4 * sum w^2 of the current weights."""
        with torch.cuda.device(self.device):
            check(lib().mpo_dn_penalty(self._h, ptr(self._pen), _lib.stream_handle(self.device)), "mpo_dn_penalty")
        return self._pen

    # -- full k-fold training -----------------------------------------------------
    def fit_folds(self, x, labels, folds, n_fold, epochs, record_train_loss=False, holdout=None, progress=None,
                  stopping=None):
        """Train every member for ``epochs`` on its fold (in order, no shuffle),
        validating once per epoch; val_loss = mean CE + l2 penalty (Keras).  The
        loop is population.train_folds."""
        return train_folds(self, x, labels, folds, n_fold, epochs, record_train_loss, holdout, progress, stopping,
                           val_offset=self.penalty)


def synthetic_cifar(n=50000, img_dim=(32, 32, 3), classes=10, seed=0, device=None):
    """CIFAR-10-shape synthetic data: x ~ U[0,1] f32 [n,H,W,C] (NHWC),
    labels uniform in [0, classes), generated on device."""
    dev = torch.device(device if device is not None else "cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    x = torch.rand((n,) + tuple(img_dim), generator=g, device=dev, dtype=torch.float32)
    y = torch.randint(0, classes, (n,), generator=g, device=dev, dtype=torch.int32)
    return x, y
