"""Device-resident population engine for MNIST-CNN trials.

Replaces the ``process_block`` / ``mpi_learn`` block-master + worker ranks
(/root/reference/process_block.py:71-96, 104-121): instead of one MPI block per
candidate network, every (trial, fold) pair is a *member* of one population
that trains on a single GPU in lock-step, ragged widths and all, through
``libmpo.so`` (csrc/cnn.hip).  torch only owns the device arenas.

Public surface:

* :class:`TrialSpec` -- test_mnist hyper-parameters + per-trial lr / dropout;
* :class:`PopulationEngine` -- low level: ``train_step`` / ``eval_step`` on
  caller-supplied batch orders (the k-fold index gather);
* :func:`kfold_split` -- the fold split (contiguous KFold, no shuffle);
* :meth:`PopulationEngine.fit_folds` -- full training of every member over
  ``epochs`` with a validation pass per epoch; returns per-member histories.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr

IMG = 28
NUM_CLASSES = 10
PARAM_NAMES = ("w1", "b1", "w2", "b2", "w3", "b3", "w4", "b4")
ACT_NAMES = ("a1", "a2", "pd", "am", "h", "hd", "z3", "dz3", "dh", "dp", "dz2", "dz1", "w2t", "wp1", "wp2")


@dataclass
class TrialSpec:
    """One test_mnist trial (mpiLAPI.py:138-176; space option3:127-131)."""

    nb_filters: int = 32
    kernel_size: int = 3
    pool_size: int = 2
    dense: int = 128
    lr: float = 1e-3
    dropout: float = 0.25
    seed: int = 0
    loss: str = "binary_crossentropy"     # option3 --loss (:61)
    optimizer: str = "adam"               # option3 --optimizer (:60), the master's update rule

    def options(self):
        """MpoCnnSpec.options bits; raises for a loss / optimizer the kernels do not implement."""
        try:
            return _lib.LOSS_CODES[self.loss] | _lib.OPT_CODES[self.optimizer]
        except KeyError:
            raise ValueError(f"unsupported loss / optimizer {self.loss!r} / {self.optimizer!r}: the population "
                             f"kernels implement losses {sorted(_lib.LOSS_CODES)} and optimizers "
                             f"{sorted(_lib.OPT_CODES)}") from None

    def geometry(self):
        H1 = IMG - self.kernel_size + 1
        H2 = H1 - self.kernel_size + 1
        s = H2 // self.pool_size
        return dict(H1=H1, H2=H2, s=s, K1=s * s * self.nb_filters)

    def param_shapes(self):
        F, k, D = self.nb_filters, self.kernel_size, self.dense
        K1 = self.geometry()["K1"]
        return {"w1": (k, k, 1, F), "b1": (F,), "w2": (k, k, F, F), "b2": (F,),
                "w3": (K1, D), "b3": (D,), "w4": (D, NUM_CLASSES), "b4": (NUM_CLASSES,)}

    def flops_per_sample_fwd(self):
        F, k, D = self.nb_filters, self.kernel_size, self.dense
        g = self.geometry()
        return 2 * k * k * F * g["H1"] ** 2 + 2 * k * k * F * F * g["H2"] ** 2 + 2 * g["K1"] * D + 2 * D * NUM_CLASSES

    def flops_per_sample_train(self):
        k, F = self.kernel_size, self.nb_filters
        return 3 * self.flops_per_sample_fwd() - 2 * k * k * F * self.geometry()["H1"] ** 2

    def hbm_bytes_train(self, batch):
        """Algorithmic HBM bytes of one train step of this member over ``batch``
        samples: the layer-by-layer schedule with every tensor written once and
        read once per consuming kernel (f32).  Per sample: x read by conv1 fwd and
        wgrad; a1 written, read by conv2 fwd / conv2 wgrad / dgrad's ReLU mask;
        a2 written and read by the pool; dz2 written, read by conv2 wgrad and
        dgrad; dz1 written, read by conv1 wgrad; the pooled / dense activations
        and their gradients (K1, dense, 10) written and read twice.  Per member:
        weights read twice (fwd, bwd), gradient written and read, Adam m, v read
        and written, weights written."""
        F, D = self.nb_filters, self.dense
        g = self.geometry()
        a1, a2, K1 = g["H1"] ** 2 * F, g["H2"] ** 2 * F, g["K1"]
        per_sample = 2 * IMG * IMG + 4 * a1 + 2 * a2 + 3 * a2 + 2 * a1 + 3 * 2 * (K1 + D + NUM_CLASSES)
        n_params = sum(int(np.prod(s)) for s in self.param_shapes().values())
        return 4 * (batch * per_sample + 8 * n_params)


    def hbm_bytes_train_by_kernel(self, batch, spg=(4, 2)):
        """Each csrc/cnn.hip kernel family's own minimal HBM bytes for one train step
        of this member (f32; every operand read once and every result written once
        per launch, as ``mpo_pop_train_step`` launches them).  Beyond
        :meth:`hbm_bytes_train` it keeps the traffic the algorithm's kernel split
        implies: the weight gradients' partial slabs (one per ``spg`` samples,
        written by the wgrad kernels, read by ``wgrad_reduce``) and ``flip_w2``'s
        padded / rotated weight copies.  Returns {family: bytes}."""
        F, D, k = self.nb_filters, self.dense, self.kernel_size
        g = self.geometry()
        a1, a2, K1 = g["H1"] ** 2 * F, g["H2"] ** 2 * F, g["K1"]
        img = IMG * IMG
        n_params = sum(int(np.prod(s)) for s in self.param_shapes().values())
        g1, g2 = -(-batch // spg[0]), -(-batch // spg[1])
        slab1, slab2 = g1 * (k * k + 1) * F, g2 * (k * k * F + 1) * F
        per = {
            "conv_img_kernel": batch * ((img + a1) + (a1 + a2)),                   # conv1, conv2 forward
            "pool_fwd_kernel": batch * (a2 + K1 + K1 / 4),                         # a2 in; pooled + u8 argmax out
            "dense_kernel": batch * (K1 + 2 * D + D + NUM_CLASSES                  # D1, D2 forward
                                     + D + NUM_CLASSES + NUM_CLASSES + 2 * D        # D2 wgrad, dgrad (+ gates)
                                     + K1 + D + D + K1),                            # D1 wgrad, dgrad
            "softmax_bce_kernel": batch * 2 * NUM_CLASSES,
            "pool_bwd_kernel": batch * (K1 + K1 / 4 + a2 + a2),                     # dp, argmax, a2 mask in; dz2 out
            "conv_wgrad_kernel": batch * (a1 + a2) + slab2,                        # a1, dz2 in; slabs out
            "conv_dgrad_kernel": batch * (a2 + a1 + a1),                           # dz2, a1 mask in; dz1 out
            "conv1_wgrad_kernel": batch * (img + a1) + slab1,
            "wgrad_reduce_kernel": slab1 + slab2 + (k * k + 1) * F + (k * k * F + 1) * F,
            "flip_w2_kernel": 3 * k * k * F * F + k * k * F,                       # w2 (w1) in; padded + rotated out
            "adam_kernel": 7 * n_params,                                            # p, g, m, v in; p, m, v out
        }
        return {name: 4.0 * v for name, v in per.items()}


MpoCnnSpec = _lib.MpoCnnSpec
MpoPopSizes = _lib.MpoPopSizes


def glorot_uniform_init(spec: TrialSpec, seed: int):
    """Keras defaults: glorot_uniform kernels, zero biases (float32)."""
    rng = np.random.RandomState(seed)
    out = {}
    for name, shape in spec.param_shapes().items():
        if name.startswith("w"):
            if len(shape) == 4:
                rf = shape[0] * shape[1]
                fan_in, fan_out = rf * shape[2], rf * shape[3]
            else:
                fan_in, fan_out = shape
            lim = np.sqrt(6.0 / (fan_in + fan_out))
            out[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
        else:
            out[name] = np.zeros(shape, dtype=np.float32)
    return out


def kfold_split(n_samples: int, n_fold: int, fold: int, holdout=None):
    """Fold split as an index gather.

    n_fold == 1 mirrors option3's file split: training on the first 70 % (of the
    files, hyperparameter_search_option3.py:136-139; of the samples when the data
    is synthetic), validation on the rest -- ``holdout`` = the number of training
    samples when they come from the train_list files.  n_fold > 1 is a contiguous
    KFold without shuffle over the training samples (the first ``holdout``, all
    if None): fold sizes n//k (+1 for the first n%k folds)."""
    idx = np.arange(n_samples, dtype=np.int32)
    if n_fold <= 1:
        cut = int(n_samples * 0.70) if holdout is None else int(holdout)
        return idx[:cut], idx[cut:]
    if holdout is not None:
        idx = idx[:int(holdout)]
        n_samples = len(idx)
    sizes = np.full(n_fold, n_samples // n_fold, dtype=np.int64)
    sizes[: n_samples % n_fold] += 1
    starts = np.concatenate([[0], np.cumsum(sizes)])
    v0, v1 = starts[fold], starts[fold + 1]
    return np.concatenate([idx[:v0], idx[v1:]]), idx[v0:v1]


class PopulationEngine:
    """A population of ragged CNN members resident on one GPU."""

    def __init__(self, specs, batch=100, device=None, init=None, init_seed=0):
        self.specs = [s if isinstance(s, TrialSpec) else TrialSpec(**s) for s in specs]
        self.n = len(self.specs)
        self.batch = int(batch)
        self.device = torch.device(device if device is not None else "cuda")
        L = lib()
        arr = (MpoCnnSpec * self.n)()
        for i, s in enumerate(self.specs):
            arr[i] = MpoCnnSpec(int(s.nb_filters), int(s.kernel_size), int(s.pool_size), int(s.dense),
                                float(s.lr), float(s.dropout), int(s.seed) & 0xFFFFFFFF, s.options())
        h = ctypes.c_void_p()
        check(L.mpo_pop_create(arr, self.n, self.batch, ctypes.byref(h)), "mpo_pop_create")
        self._h = h
        sz = MpoPopSizes()
        check(L.mpo_pop_sizes(h, ctypes.byref(sz)), "mpo_pop_sizes")
        self.n_params = int(sz.n_params)
        self.layout = []
        offs = (ctypes.c_int64 * 9)()
        for i in range(self.n):
            check(L.mpo_pop_param_layout(h, i, offs), "mpo_pop_param_layout")
            self.layout.append([int(v) for v in offs])
        self.act_layout = []
        aoffs = (ctypes.c_int64 * 15)()
        for i in range(self.n):
            check(L.mpo_pop_act_layout(h, i, aoffs), "mpo_pop_act_layout")
            self.act_layout.append(dict(zip(ACT_NAMES, [int(v) for v in aoffs])))
        dev = self.device
        self.params = torch.zeros(self.n_params, dtype=torch.float32, device=dev)
        self.grads = torch.zeros_like(self.params)
        self.adam_m = torch.zeros_like(self.params)
        self.adam_v = torch.zeros_like(self.params)
        self.act = torch.zeros(int(sz.act_floats), dtype=torch.float32, device=dev)
        self.tables = torch.empty(int(sz.table_bytes), dtype=torch.uint8, device=dev)
        self.loss = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.val_loss_sum = torch.zeros(self.n, dtype=torch.float32, device=dev)
        self.val_correct = torch.zeros(self.n, dtype=torch.int32, device=dev)
        with torch.cuda.device(dev):
            check(L.mpo_pop_bind(h, ptr(self.params), ptr(self.grads), ptr(self.adam_m), ptr(self.adam_v),
                                 ptr(self.act), ptr(self.tables), _lib.stream_handle(dev)), "mpo_pop_bind")
        if init is None:
            init = [glorot_uniform_init(s, init_seed + i) for i, s in enumerate(self.specs)]
        for i, p in enumerate(init):
            self.set_params(i, p)
        self.step_count = 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().mpo_pop_destroy(h)
            except Exception:
                pass
            self._h = None

    # -- parameters -------------------------------------------------------------
    def _slices(self, i):
        o = self.layout[i]
        shapes = self.specs[i].param_shapes()
        return {n: (o[j], shapes[n]) for j, n in enumerate(PARAM_NAMES)}

    def set_params(self, i, params):
        flat = []
        for n, (off, shape) in self._slices(i).items():
            a = np.asarray(params[n], dtype=np.float32).reshape(shape)
            cnt = int(np.prod(shape))
            self.params[off:off + cnt].copy_(torch.from_numpy(a.reshape(-1)))
            flat.append(cnt)

    def get_params(self, i):
        out = {}
        host = self.params.cpu().numpy()
        for n, (off, shape) in self._slices(i).items():
            cnt = int(np.prod(shape))
            out[n] = host[off:off + cnt].reshape(shape).copy()
        return out

    def activation(self, i, name, shape):
        """Copy of member i's activation tensor ``name`` (diagnostics / tests)."""
        off = self.act_layout[i][name]
        cnt = int(np.prod(shape))
        return self.act[off:off + cnt].reshape(shape).cpu().numpy()

    def argmax_table(self, i):
        """Member i's max-pool argmax (uint8, [batch, s*s*F]) of the last forward."""
        K1 = self.specs[i].geometry()["K1"]
        off = self.act_layout[i]["am"] * 4
        n = self.batch * K1
        raw = self.act.view(torch.uint8)[off:off + n]
        return raw.cpu().numpy().reshape(self.batch, K1)

    def reset_optimizer(self):
        self.adam_m.zero_()
        self.adam_v.zero_()
        self.step_count = 0

    # -- steps --------------------------------------------------------------------
    def train_step(self, x, labels, order, row0, step=None):
        """x [n,784] f32, labels [n] i32, order [n_members, L] i32 (device)."""
        step = self.step_count if step is None else int(step)
        with torch.cuda.device(self.device):
            check(lib().mpo_pop_train_step(self._h, ptr(x), ptr(labels), ptr(order), int(order.shape[1]), int(row0),
                                           step, ptr(self.loss), _lib.stream_handle(self.device)),
                  "mpo_pop_train_step")
        self.step_count = step + 1
        return self.loss

    def profile(self, reset=True):
        """Per-phase device ms since the last reset ({phase: ms}); empty unless the
        engine was created with MPO_POP_PROFILE=1 in the environment."""
        buf = ctypes.create_string_buffer(8192)
        rc = lib().mpo_pop_profile(self._h, buf, len(buf), int(reset))
        if rc != _lib.MPO_OK:
            return {}
        out = {}
        for line in buf.value.decode().splitlines():
            name, ms = line.split()
            out[name] = float(ms)
        return out

    def eval_reset(self):
        self.val_loss_sum.zero_()
        self.val_correct.zero_()

    def eval_step(self, x, labels, order, row0):
        with torch.cuda.device(self.device):
            check(lib().mpo_pop_eval_step(self._h, ptr(x), ptr(labels), ptr(order), int(order.shape[1]), int(row0),
                                          ptr(self.val_loss_sum), ptr(self.val_correct),
                                          _lib.stream_handle(self.device)), "mpo_pop_eval_step")

    # -- full k-fold training -----------------------------------------------------
    def fit_folds(self, x, labels, folds, n_fold, epochs, record_train_loss=False, holdout=None, progress=None,
                  stopping=None):
        """Train every member for ``epochs`` on its fold's training indices (in
        order, no shuffle), validating once per epoch (validate_every =
        count/batch, option3:260).  ``folds[i]`` is member i's fold index;
        ``progress(epoch, epochs)`` is called after each epoch's validation;
        ``stopping`` (a :class:`~mpi_opt_amd.stopping.StopRule`) ends members early.
        Returns {"val_loss": [n, epochs], "val_acc": [n, epochs], "epochs_run": [n], ...}."""
        return train_folds(self, x, labels, folds, n_fold, epochs, record_train_loss, holdout, progress, stopping)


def train_folds(eng, x, labels, folds, n_fold, epochs, record_train_loss=False, holdout=None, progress=None,
                stopping=None, val_offset=None):
    """The k-fold training loop shared by the MNIST and DenseNet populations
    (``eng.train_step`` / ``eval_reset`` / ``eval_step`` / ``val_loss_sum`` /
    ``val_correct``): members step in lock-step on full batches, every member on
    the first steps_per_epoch*B indices of its fold, validating on the first
    val_batches*B; what that leaves out (uneven folds, a partial last batch that
    Keras would still run) is reported in the history, never hidden.
    ``val_offset()`` is added to the validation loss (DenseNet's l2 penalty)."""
    n_samples = x.shape[0]
    B = eng.batch
    tr, va = [], []
    for i in range(eng.n):
        t, v = kfold_split(n_samples, n_fold, int(folds[i]), holdout)
        tr.append(t)
        va.append(v)
    n_tr = min(len(t) for t in tr)
    n_va = min(len(v) for v in va)
    steps_per_epoch = n_tr // B
    val_batches = n_va // B
    if steps_per_epoch == 0 or val_batches == 0:
        raise ValueError(f"fold too small for batch {B}: {n_tr} train / {n_va} validation samples")
    dropped_tr = [len(t) - steps_per_epoch * B for t in tr]
    dropped_va = [len(v) - val_batches * B for v in va]
    order_tr = torch.from_numpy(np.stack([t[:n_tr] for t in tr])).to(eng.device)
    order_va = torch.from_numpy(np.stack([v[:n_va] for v in va])).to(eng.device)
    val_loss = torch.zeros(eng.n, epochs, dtype=torch.float32, device=eng.device)
    val_acc = torch.zeros(eng.n, epochs, dtype=torch.float32, device=eng.device)
    state = stopping.start(eng.n) if stopping is not None else None
    tl = []
    for ep in range(epochs):
        for st in range(steps_per_epoch):
            loss = eng.train_step(x, labels, order_tr, st * B)
            if record_train_loss:
                tl.append(loss.clone())
        eng.eval_reset()
        for vb in range(val_batches):
            eng.eval_step(x, labels, order_va, vb * B)
        denom = float(val_batches * B)
        val_loss[:, ep] = eng.val_loss_sum / denom + (val_offset() if val_offset is not None else 0.0)
        val_acc[:, ep] = eng.val_correct.to(torch.float32) / denom
        if progress is not None:
            progress(ep + 1, epochs)
        if state is not None:
            state.update(ep, val_loss[:, ep].cpu().numpy(), val_acc[:, ep].cpu().numpy())
            if state.all_stopped():
                break
    out = {"val_loss": val_loss.cpu().numpy(), "val_acc": val_acc.cpu().numpy(),
           "steps_per_epoch": steps_per_epoch, "val_batches": val_batches,
           "dropped_train_samples": dropped_tr, "dropped_val_samples": dropped_va,
           "epochs_run": state.epochs(epochs) if state is not None else np.full(eng.n, epochs)}
    if record_train_loss:
        out["train_loss"] = torch.stack(tl, 1).cpu().numpy() if tl else np.zeros((eng.n, 0))
    return out


def kfold_gather(X, idx, out=None):
    """``mpo_kfold_gather``: out[r] = X[idx[r]] on device."""
    rows = idx.shape[0]
    row_elems = int(np.prod(X.shape[1:]))
    if out is None:
        out = torch.empty((rows,) + tuple(X.shape[1:]), dtype=X.dtype, device=X.device)
    with torch.cuda.device(X.device):
        check(lib().mpo_kfold_gather(ptr(X), ptr(idx), int(rows), row_elems, ptr(out),
                                     _lib.stream_handle(X.device)), "mpo_kfold_gather")
    return out


def synthetic_mnist(n=60000, seed=0, device=None, labels="uniform"):
    """x ~ U[0,1] f32 (n, 784), generated on device.

    ``labels="uniform"``: labels uniform 0..9 (§8d; nothing to learn, so every
    trial's validation loss is the uniform-softmax BCE and a search sees a flat
    objective).  ``labels="learnable"``: the label of an image is the argmax of a
    fixed random linear teacher over its 4x4-average-pooled 7x7 image, centred at
    0.5 -- a function a test_mnist CNN learns, so trials differ by their
    hyper-parameters and the GP of a search fits a non-flat objective."""
    g = torch.Generator(device=device if device is not None else "cuda")
    g.manual_seed(seed)
    dev = torch.device(device if device is not None else "cuda")
    x = torch.rand(n, IMG * IMG, generator=g, device=dev, dtype=torch.float32)
    y = torch.randint(0, NUM_CLASSES, (n,), generator=g, device=dev, dtype=torch.int32)
    if labels == "learnable":
        w = torch.randn(49, NUM_CLASSES, generator=g, device=dev, dtype=torch.float32)
        pooled = x.view(n, 7, 4, 7, 4).mean(dim=(2, 4)).reshape(n, 49) - 0.5
        y = torch.argmax(pooled @ w, dim=1).to(torch.int32)
    elif labels != "uniform":
        raise ValueError(f"labels {labels!r}: 'uniform' or 'learnable'")
    return x, y
