"""CPU oracle for the DenseNet population.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker; the product (``mpi_opt_amd``) never imports it.

What it restates (numpy, float64)
---------------------------------
``DenseNet(nb_classes, img_dim, depth, nb_dense_block, growth_rate, nb_filter,
dropout_rate=0, weight_decay=1e-4)`` (/root/reference/densenet.py:135-196) with
``conv_factory`` (:12-37), ``transition`` (:40-67) and ``denseblock`` (:70-100),
compiled with ``Adam(lr)`` + ``categorical_crossentropy``
(/root/reference/base_model.py:61-72, mpiLAPI.py:197-201), channels-last input:

    x -> Conv3x3(nb_filter, same, no bias)                          [initial_conv2D]
    per block: (depth-4)/3 x [ BN(axis=1) -> ELU -> Conv3x3(growth, same, no bias) ]
               each output concatenated on the channel axis (concat_axis=-1)
    between blocks: BN(axis=1) -> ELU -> Conv1x1(C, no bias) -> AvgPool(2, 2)
    BN(axis=1) -> ELU -> GlobalAveragePooling -> Dense(nb_classes) -> softmax

Keras semantics kept:
* ``BatchNormalization(mode=0, axis=1)`` on an NHWC tensor normalises over
  (batch, W, C) **per image row** -- gamma/beta/moving stats have shape [H]
  (the "axis=1 quirk", densenet.py:24-27).  Training uses the batch mean and the
  biased batch variance, epsilon 1e-3; the moving averages update with momentum
  0.99; evaluation uses the moving averages.  Keras' moving-variance update is
  version dependent (unbiased from Keras 2.1.3); Keras is absent and unpinned,
  so the biased batch variance is used -- "parity unpinned" for that detail.
* ELU(alpha=1) = x if x > 0 else expm1(x); he_uniform kernels (init is made by
  the caller and passed in); gamma = 1, beta = 0, moving mean 0 / var 1.
* l2(1e-4) on every conv kernel, every gamma/beta and the dense kernel + bias:
  the loss adds 1e-4 * sum(w^2), the gradient 2e-4 * w.
* categorical cross-entropy on softmax: p /= sum(p), clip(p, 1e-7, 1 - 1e-7),
  -sum(onehot * log p), batch mean; the clipped target has zero gradient.
* Adam(lr, b1=.9, b2=.999, eps=1e-8) in Keras' bias-corrected-lr form, one
  update per batch (the same mpi_learn single-trial restatement as oracle/cnn.py).
* dropout_rate is 0 in the reference's search grid (base_model.py:84-92) and is
  not modelled.
"""
from __future__ import annotations

import numpy as np

BN_EPS = 1e-3
BN_MOMENTUM = 0.99
L2 = 1e-4
CE_EPS = 1e-7


# --- architecture -----------------------------------------------------------
def arch_layers(img_dim=(32, 32, 3), nb_classes=10, depth=10, nb_dense_block=3, growth_rate=12, nb_filter=16):
    """Layer list of DenseNet (densenet.py:155-196) as dicts with the stage
    geometry; parameter names in Keras creation order."""
    assert (depth - 4) % 3 == 0, "Depth must be 3 N + 4"
    H, W, C0 = img_dim
    L = (depth - 4) // 3
    layers = [dict(kind="conv0", H=H, W=W, cin=C0, cout=nb_filter, ks=3, coff=0)]
    f = nb_filter
    stage = 0
    for blk in range(nb_dense_block):
        for _ in range(L):
            layers.append(dict(kind="dense", stage=stage, H=H, W=W, cin=f, cout=growth_rate, ks=3, coff=f))
            f += growth_rate
        if blk < nb_dense_block - 1:
            layers.append(dict(kind="trans", stage=stage, H=H, W=W, cin=f, cout=f, ks=1, coff=0))
            H, W = H // 2, W // 2
            stage += 1
    layers.append(dict(kind="head", stage=stage, H=H, W=W, cin=f, cout=nb_classes))
    return layers


def stage_dims(layers):
    """[(H, W, C_total)] of each concat stage."""
    out = {}
    for ly in layers:
        if ly["kind"] in ("dense", "trans", "head"):
            s = ly["stage"]
            out[s] = (ly["H"], ly["W"], max(out.get(s, (0, 0, 0))[2], ly["cin"] + (ly["cout"] if ly["kind"] == "dense" else 0)))
    return [out[s] for s in sorted(out)]


def param_shapes(layers):
    """Trainable tensors (Keras order) and BN moving-stat shapes."""
    P, S = {}, {}
    for i, ly in enumerate(layers):
        if ly["kind"] == "conv0":
            P[f"w{i}"] = (3, 3, ly["cin"], ly["cout"])
        elif ly["kind"] in ("dense", "trans"):
            P[f"g{i}"] = (ly["H"],)
            P[f"b{i}"] = (ly["H"],)
            P[f"w{i}"] = (ly["ks"], ly["ks"], ly["cin"], ly["cout"])
            S[f"mm{i}"] = (ly["H"],)
            S[f"mv{i}"] = (ly["H"],)
        else:
            P[f"g{i}"] = (ly["H"],)
            P[f"b{i}"] = (ly["H"],)
            P[f"wd"] = (ly["cin"], ly["cout"])
            P[f"bd"] = (ly["cout"],)
            S[f"mm{i}"] = (ly["H"],)
            S[f"mv{i}"] = (ly["H"],)
    return P, S


def flops_per_sample_fwd(layers):
    tot = 0
    for ly in layers:
        if ly["kind"] == "head":
            tot += 2 * ly["cin"] * ly["cout"]
        else:
            tot += 2 * ly["ks"] ** 2 * ly["cin"] * ly["cout"] * ly["H"] * ly["W"]
    return tot


def flops_per_sample_train(layers):
    """fwd + dgrad + wgrad of every conv/dense, minus the initial conv's dgrad."""
    c0 = layers[0]
    return 3 * flops_per_sample_fwd(layers) - 2 * 9 * c0["cin"] * c0["cout"] * c0["H"] * c0["W"]


# --- ops ----------------------------------------------------------------------
def _pad(x, p):
    return np.pad(x, ((0, 0), (p, p), (p, p), (0, 0))) if p else x


def _im2col(x, ks):
    """x [B,H,W,C] -> [B*H*W, ks*ks*C] for a stride-1 'same' conv, (ky,kx,c) order."""
    B, H, W, C = x.shape
    xp = _pad(x, (ks - 1) // 2)
    cols = np.empty((B, H, W, ks, ks, C), dtype=x.dtype)
    for ky in range(ks):
        for kx in range(ks):
            cols[:, :, :, ky, kx, :] = xp[:, ky:ky + H, kx:kx + W, :]
    return cols.reshape(B * H * W, ks * ks * C)


def conv_same(x, w):
    B, H, W, _ = x.shape
    ks, _, cin, cout = w.shape
    return (_im2col(x, ks) @ w.reshape(-1, cout)).reshape(B, H, W, cout)


def conv_same_bwd(dout, x, w, need_dx=True):
    B, H, W, cout = dout.shape
    ks, _, cin, _ = w.shape
    d2 = dout.reshape(-1, cout)
    dw = (_im2col(x, ks).T @ d2).reshape(w.shape)
    dx = None
    if need_dx:
        # 'same' stride-1 conv transpose = 'same' conv with the rotated, transposed kernel
        wt = w[::-1, ::-1].transpose(0, 1, 3, 2)
        dx = conv_same(dout, np.ascontiguousarray(wt))
    return dx, dw


def bn_elu_fwd(x, gamma, beta, train, mm, mv):
    """BN(axis=1 of NHWC: per image row) -> ELU.  Returns z and the cache."""
    if train:
        mean = x.mean(axis=(0, 2, 3))
        var = x.var(axis=(0, 2, 3))
    else:
        mean, var = mm, mv
    inv = 1.0 / np.sqrt(var + BN_EPS)
    xhat = (x - mean[None, :, None, None]) * inv[None, :, None, None]
    y = gamma[None, :, None, None] * xhat + beta[None, :, None, None]
    z = np.where(y > 0, y, np.expm1(np.minimum(y, 0)))
    return z, dict(xhat=xhat, inv=inv, y=y, mean=mean, var=var)


def bn_elu_bwd(dz, gamma, c):
    dy = dz * np.where(c["y"] > 0, 1.0, np.exp(np.minimum(c["y"], 0)))
    xhat, inv = c["xhat"], c["inv"]
    n = dy.shape[0] * dy.shape[2] * dy.shape[3]
    dbeta = dy.sum(axis=(0, 2, 3))
    dgamma = (dy * xhat).sum(axis=(0, 2, 3))
    dx = (gamma * inv / n)[None, :, None, None] * (n * dy - dbeta[None, :, None, None]
                                                  - xhat * dgamma[None, :, None, None])
    return dx, dgamma, dbeta


def avgpool2(x):
    B, H, W, C = x.shape
    H2, W2 = H // 2, W // 2
    v = x[:, :2 * H2, :2 * W2, :].reshape(B, H2, 2, W2, 2, C)
    return v.mean(axis=(2, 4))


def avgpool2_bwd(d, shape):
    B, H, W, C = shape
    H2, W2 = d.shape[1], d.shape[2]
    out = np.zeros(shape, dtype=d.dtype)
    up = np.repeat(np.repeat(d, 2, axis=1), 2, axis=2) * 0.25
    out[:, :2 * H2, :2 * W2, :] = up
    return out


def softmax(z):
    e = np.exp(z - z.max(axis=1, keepdims=True))
    return e / e.sum(axis=1, keepdims=True)


def cce_loss_and_grad(logits, onehot):
    """Keras categorical_crossentropy on softmax output: per-sample loss and d/dlogits
    of the batch mean."""
    p = softmax(logits)
    p = p / p.sum(axis=1, keepdims=True)
    pc = np.clip(p, CE_EPS, 1 - CE_EPS)
    loss = -(onehot * np.log(pc)).sum(axis=1)
    pt = (p * onehot).sum(axis=1)
    live = ((pt >= CE_EPS) & (pt <= 1 - CE_EPS)).astype(p.dtype)
    dlogits = (p - onehot) * live[:, None] / logits.shape[0]
    return loss, dlogits


def he_uniform_init(layers, seed):
    """Keras he_uniform kernels (limit sqrt(6 / fan_in)), glorot-uniform dense
    kernel, zero biases, gamma 1 / beta 0, moving mean 0 / var 1 (float64)."""
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
    return params, state


# --- model --------------------------------------------------------------------
class DenseNetOracle:
    """One DenseNet trial trained single-process in float64."""

    def __init__(self, layers, params, state=None, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8):
        self.layers = layers
        self.params = {k: np.array(v, dtype=np.float64) for k, v in params.items()}
        P, S = param_shapes(layers)
        if state is None:
            state = {n: (np.zeros(s) if n.startswith("mm") else np.ones(s)) for n, s in S.items()}
        self.state = {k: np.array(v, dtype=np.float64) for k, v in state.items()}
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        self.m = {k: np.zeros_like(v) for k, v in self.params.items()}
        self.v = {k: np.zeros_like(v) for k, v in self.params.items()}
        self.t = 0

    def l2_penalty(self):
        return L2 * sum(float((v * v).sum()) for v in self.params.values())

    def forward(self, x, y, train=True):
        """x [B,H,W,C] (float), y [B] int.  Returns (mean CE + l2, per-sample CE,
        predictions, cache)."""
        P, S = self.params, self.state
        ls = self.layers
        B = x.shape[0]
        x = np.asarray(x, dtype=np.float64)
        cache = {"x": x}
        cat = None
        for i, ly in enumerate(ls):
            k = ly["kind"]
            if k == "conv0":
                H, W = ly["H"], ly["W"]
                C = _stage_c(ls, 0)
                cat = np.zeros((B, H, W, C))
                cat[..., :ly["cout"]] = conv_same(x, P[f"w{i}"])
            elif k == "dense":
                xin = cat[..., :ly["cin"]].copy()
                z, c = bn_elu_fwd(xin, P[f"g{i}"], P[f"b{i}"], train, S[f"mm{i}"], S[f"mv{i}"])
                cache[i] = (z, c)
                cat[..., ly["coff"]:ly["coff"] + ly["cout"]] = conv_same(z, P[f"w{i}"])
            elif k == "trans":
                xin = cat[..., :ly["cin"]].copy()
                z, c = bn_elu_fwd(xin, P[f"g{i}"], P[f"b{i}"], train, S[f"mm{i}"], S[f"mv{i}"])
                t = conv_same(z, P[f"w{i}"])
                cache[i] = (z, c, t.shape)
                pooled = avgpool2(t)
                cache[("cat", ly["stage"])] = cat
                cat = np.zeros(pooled.shape[:3] + (_stage_c(ls, ly["stage"] + 1),))
                cat[..., :ly["cout"]] = pooled
            else:
                xin = cat[..., :ly["cin"]]
                z, c = bn_elu_fwd(xin, P[f"g{i}"], P[f"b{i}"], train, S[f"mm{i}"], S[f"mv{i}"])
                g = z.mean(axis=(1, 2))
                logits = g @ P["wd"] + P["bd"]
                cache[i] = (z, c, g)
                cache[("cat", ly["stage"])] = cat
        onehot = np.eye(ls[-1]["cout"])[np.asarray(y)]
        ce, dlogits = cce_loss_and_grad(logits, onehot)
        cache["dlogits"] = dlogits
        if train:
            for i, ly in enumerate(ls):
                if ly["kind"] != "conv0":
                    c = cache[i][1]
                    S[f"mm{i}"] = BN_MOMENTUM * S[f"mm{i}"] + (1 - BN_MOMENTUM) * c["mean"]
                    S[f"mv{i}"] = BN_MOMENTUM * S[f"mv{i}"] + (1 - BN_MOMENTUM) * c["var"]
        loss = float(ce.mean()) + self.l2_penalty()
        return loss, ce, logits.argmax(axis=1), cache

    def backward(self, cache):
        P = self.params
        ls = self.layers
        grads = {}
        dcat = None
        for i in range(len(ls) - 1, -1, -1):
            ly = ls[i]
            k = ly["kind"]
            if k == "head":
                z, c, g = cache[i]
                dl = cache["dlogits"]
                grads["wd"] = g.T @ dl
                grads["bd"] = dl.sum(0)
                dg = dl @ P["wd"].T
                H, W = ly["H"], ly["W"]
                dz = np.broadcast_to(dg[:, None, None, :] / (H * W), z.shape)
                dx, grads[f"g{i}"], grads[f"b{i}"] = bn_elu_bwd(dz, P[f"g{i}"], c)
                cat = cache[("cat", ly["stage"])]
                dcat = np.zeros(cat.shape)
                dcat[..., :ly["cin"]] += dx
            elif k == "trans":
                z, c, tshape = cache[i]
                dpool = dcat[..., :ly["cout"]]
                dt = avgpool2_bwd(dpool, tshape)
                dz, grads[f"w{i}"] = conv_same_bwd(dt, z, P[f"w{i}"])
                dx, grads[f"g{i}"], grads[f"b{i}"] = bn_elu_bwd(dz, P[f"g{i}"], c)
                cat = cache[("cat", ly["stage"])]
                dcat = np.zeros(cat.shape)
                dcat[..., :ly["cin"]] += dx
            elif k == "dense":
                z, c = cache[i]
                dout = dcat[..., ly["coff"]:ly["coff"] + ly["cout"]]
                dz, grads[f"w{i}"] = conv_same_bwd(dout, z, P[f"w{i}"])
                dx, grads[f"g{i}"], grads[f"b{i}"] = bn_elu_bwd(dz, P[f"g{i}"], c)
                dcat[..., :ly["cin"]] += dx
            else:
                dout = dcat[..., :ly["cout"]]
                _, grads[f"w{i}"] = conv_same_bwd(dout, cache["x"], P[f"w{i}"], need_dx=False)
        for n in grads:
            grads[n] = grads[n] + 2 * L2 * P[n]
        return grads

    def adam(self, grads):
        self.t += 1
        t = self.t
        lr_t = self.lr * np.sqrt(1.0 - self.b2 ** t) / (1.0 - self.b1 ** t)
        for n in self.params:
            gr = grads[n]
            self.m[n] = self.b1 * self.m[n] + (1 - self.b1) * gr
            self.v[n] = self.b2 * self.v[n] + (1 - self.b2) * gr * gr
            self.params[n] = self.params[n] - lr_t * self.m[n] / (np.sqrt(self.v[n]) + self.eps)

    def train_step(self, x, y):
        loss, _, _, cache = self.forward(x, y, train=True)
        self.adam(self.backward(cache))
        return loss

    def eval_batch(self, x, y):
        """(sum of per-sample CE, correct count) in inference mode."""
        _, ce, pred, _ = self.forward(x, y, train=False)
        return float(ce.sum()), int((pred == np.asarray(y)).sum())


def _stage_c(layers, stage):
    c = 0
    for ly in layers:
        if ly["kind"] in ("dense", "trans", "head") and ly["stage"] == stage:
            c = max(c, ly["cin"] + (ly["cout"] if ly["kind"] == "dense" else 0))
    return c
