"""Generate tests/golden/trajectories.npz: fp64 oracle trajectories for the long
parity cases of tests/trajectory_cases.py (run here, on the host; the GPU tests
compare the device populations against these numbers).

    python tests/golden/make_trajectory_golden.py [pop|epoch|densenet ...]

* pop:      8 sampled members of the 320-member configs[2] population, 20 train
            steps each + one validation batch pair (oracle/cnn.py);
* epoch:    2 members, one whole 5-fold fold-epoch (480 steps) + the fold's full
            validation pass (oracle/cnn.py);
* epoch_fp32: the same 480 steps by torch-CPU fp32 (oracle/cnn_torch.py), the
            envelope of fp32-vs-fp64 trajectory divergence;
* densenet: 2 DenseNets at the configs[4] geometry, batch 100, 20 steps + one
            inference-mode validation batch (oracle/densenet.py).
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import cnn as C  # noqa: E402
from oracle import densenet as OD  # noqa: E402
from tests import trajectory_cases as T  # noqa: E402

OUT = os.path.join(HERE, "trajectories.npz")


def kfold(n, k, f):
    idx = np.arange(n, dtype=np.int32)
    sizes = np.full(k, n // k)
    sizes[: n % k] += 1
    st = np.concatenate([[0], np.cumsum(sizes)])
    return np.concatenate([idx[:st[f]], idx[st[f + 1]:]]), idx[st[f]:st[f + 1]]


def oracle(m):
    F, k, p, d, lr, dr, fold, dseed, iseed = m
    init = T.glorot_init(F, k, p, d, iseed)
    return C.TrialOracle(F, k, p, d, {n: v.astype(np.float64) for n, v in init.items()}, lr=lr, dropout=dr,
                         seed=dseed)


def make_pop():
    x, y = T.pop_data()
    members = T.pop_members()
    picks = T.pop_sampled()
    losses, vals = [], []
    for i in picks:
        m = members[i]
        o = oracle(m)
        tr, va = kfold(T.POP_SAMPLES, T.POP_FOLDS, m[6])
        spe = len(tr) // T.BATCH
        ls = []
        for st in range(T.POP_STEPS):
            rows = tr[(st % spe) * T.BATCH:(st % spe + 1) * T.BATCH]
            ls.append(o.train_step(x[rows], y[rows], st))
        losses.append(ls)
        vals.append(o.eval_loss(x[va[:2 * T.BATCH]], y[va[:2 * T.BATCH]]))
        print("pop member", i, m[:6], "loss", ls[0], "->", ls[-1], flush=True)
    return {"pop_picks": np.array(picks), "pop_train_loss": np.array(losses), "pop_val_loss": np.array(vals)}


def make_epoch():
    x, y = T.epoch_data()
    losses, vals = [], []
    for m in T.EPOCH_MEMBERS:
        o = oracle(m)
        tr, va = kfold(T.EPOCH_SAMPLES, T.EPOCH_FOLDS, m[6])
        t0 = time.time()
        ls = [o.train_step(x[tr[s * T.BATCH:(s + 1) * T.BATCH]], y[tr[s * T.BATCH:(s + 1) * T.BATCH]], s)
              for s in range(len(tr) // T.BATCH)]
        losses.append(ls)
        vals.append(o.eval_loss(x[va], y[va]))
        print("epoch member", m[:6], len(ls), "steps", ls[0], "->", ls[-1], "val", vals[-1],
              f"{time.time() - t0:.0f} s", flush=True)
    return {"epoch_train_loss": np.array(losses), "epoch_val_loss": np.array(vals)}


def make_epoch_fp32():
    """The same fold-epoch trained by an INDEPENDENT fp32 implementation (torch
    CPU autograd, oracle/cnn_torch.py, same init / order / masks): how far any
    fp32 trajectory drifts from the fp64 one over 480 Adam steps."""
    import torch

    from oracle import cnn_torch as CT

    x, y = T.epoch_data()
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    losses = []
    for m in T.EPOCH_MEMBERS:
        F, k, p, d, lr, dr, fold, dseed, iseed = m
        masks = lambda step, layer, n, rate, ds=dseed: C.dropout_keep(ds, step, layer, n, rate)  # noqa: E731
        t = CT.TorchTrial(F, k, p, d, T.glorot_init(F, k, p, d, iseed), lr=lr, dropout=dr, mask_fn=masks)
        tr, _ = kfold(T.EPOCH_SAMPLES, T.EPOCH_FOLDS, fold)
        ls = []
        for s in range(len(tr) // T.BATCH):
            rows = torch.from_numpy(tr[s * T.BATCH:(s + 1) * T.BATCH].astype(np.int64))
            ls.append(t.train_step(xt[rows], yt[rows], s))
        losses.append(ls)
        print("epoch member fp32 torch", m[:6], ls[0], "->", ls[-1], flush=True)
    return {"epoch_train_loss_fp32": np.array(losses)}


def make_densenet():
    from mpi_opt_amd.densenet import he_uniform_init  # init shared with the device side

    x, y, order = T.dn_data()
    layers = OD.arch_layers()
    losses, vs, vc, mm = [], [], [], []
    for i, lr in enumerate(T.DN_LRS):
        p, s = he_uniform_init(layers, 300 + i)
        o = OD.DenseNetOracle(layers, {k: v.astype(np.float64) for k, v in p.items()},
                              {k: v.astype(np.float64) for k, v in s.items()}, lr=lr)
        ls = []
        for st in range(T.DN_STEPS):
            idx = order[i, st * T.BATCH:(st + 1) * T.BATCH]
            ls.append(o.train_step(x[idx], y[idx]))
        idx = order[i, 1500:1600]
        s_, c_ = o.eval_batch(x[idx], y[idx])
        losses.append(ls)
        vs.append(s_)
        vc.append(c_)
        mm.append(o.state["mm1"])
        print("densenet lr", lr, ls[0], "->", ls[-1], "val", s_, c_, flush=True)
    return {"dn_train_loss": np.array(losses), "dn_val_sum": np.array(vs), "dn_val_correct": np.array(vc),
            "dn_mm1": np.array(mm)}


def make_densenet32():
    """configs[4]: the sampled members of the 32-member population (init seed
    500 + member, per-member sample order), 10 steps each on the fp64 oracle."""
    from mpi_opt_amd.densenet import he_uniform_init

    x, y, _ = T.dn_data()
    order = T.dn32_order()
    layers = OD.arch_layers()
    losses = []
    for i in T.DN32_PICKS:
        p, s = he_uniform_init(layers, 500 + i)
        o = OD.DenseNetOracle(layers, {k: v.astype(np.float64) for k, v in p.items()},
                              {k: v.astype(np.float64) for k, v in s.items()}, lr=float(T.DN32_LRS[i]))
        ls = [o.train_step(x[order[i, st * T.BATCH:(st + 1) * T.BATCH]], y[order[i, st * T.BATCH:(st + 1) * T.BATCH]])
              for st in range(T.DN32_STEPS)]
        losses.append(ls)
        print("densenet32 member", i, "lr", T.DN32_LRS[i], ls[0], "->", ls[-1], flush=True)
    return {"dn32_train_loss": np.array(losses)}


if __name__ == "__main__":
    want = sys.argv[1:] or ["pop", "epoch", "epoch_fp32", "densenet", "densenet32"]
    data = dict(np.load(OUT)) if os.path.exists(OUT) else {}
    for w in want:
        data.update({"pop": make_pop, "epoch": make_epoch, "epoch_fp32": make_epoch_fp32,
                     "densenet": make_densenet, "densenet32": make_densenet32}[w]())
        np.savez(OUT, **data)
    print("wrote", OUT, sorted(data))
