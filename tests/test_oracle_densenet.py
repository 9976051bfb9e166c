"""Pins the DenseNet oracle (oracle/densenet.py) to an independent
implementation: torch CPU autograd in float64 of the same network
(densenet.py:135-196 structure, BN axis=1 on NHWC, ELU, same-padded convs,
AvgPool2, GAP, softmax + clipped categorical CE, l2 1e-4)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

from oracle import densenet as od


def torch_loss(layers, params, x, y):
    P = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in params.items()}
    xt = torch.tensor(x, dtype=torch.float64)

    def conv(z, w):  # z NHWC, w [ks,ks,cin,cout]
        ks = w.shape[0]
        out = Fn.conv2d(z.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), padding=(ks - 1) // 2)
        return out.permute(0, 2, 3, 1)

    def bn_elu(z, g, b):
        mean = z.mean(dim=(0, 2, 3), keepdim=True)
        var = ((z - mean) ** 2).mean(dim=(0, 2, 3), keepdim=True)
        y_ = (z - mean) / torch.sqrt(var + od.BN_EPS) * g[None, :, None, None] + b[None, :, None, None]
        return Fn.elu(y_)

    feats = None
    for i, ly in enumerate(layers):
        if ly["kind"] == "conv0":
            feats = [conv(xt, P[f"w{i}"])]
        elif ly["kind"] == "dense":
            cat = torch.cat(feats, dim=3)
            feats.append(conv(bn_elu(cat, P[f"g{i}"], P[f"b{i}"]), P[f"w{i}"]))
        elif ly["kind"] == "trans":
            cat = torch.cat(feats, dim=3)
            t = conv(bn_elu(cat, P[f"g{i}"], P[f"b{i}"]), P[f"w{i}"])
            feats = [Fn.avg_pool2d(t.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)]
        else:
            cat = torch.cat(feats, dim=3)
            g = bn_elu(cat, P[f"g{i}"], P[f"b{i}"]).mean(dim=(1, 2))
            logits = g @ P["wd"] + P["bd"]
    p = torch.softmax(logits, dim=1)
    p = p / p.sum(dim=1, keepdim=True)
    pc = torch.clamp(p, od.CE_EPS, 1 - od.CE_EPS)
    ce = -torch.log(pc[torch.arange(len(y)), torch.tensor(y)])
    loss = ce.mean() + od.L2 * sum((v * v).sum() for v in P.values())
    loss.backward()
    return float(loss), {k: v.grad.numpy() for k, v in P.items()}


@pytest.mark.parametrize("img,depth,blocks,B", [((8, 8, 3), 7, 3, 3), ((12, 10, 3), 10, 2, 2), ((9, 9, 2), 7, 2, 2)])
def test_oracle_matches_torch_autograd(img, depth, blocks, B):
    layers = od.arch_layers(img_dim=img, nb_classes=5, depth=depth, nb_dense_block=blocks, growth_rate=4,
                            nb_filter=6)
    params, state = od.he_uniform_init(layers, seed=3)
    rng = np.random.RandomState(1)
    # non-trivial BN affine so gamma/beta gradients are exercised away from 1/0
    for n in params:
        if n[0] in "gb" and n != "bd":
            params[n] = params[n] + 0.3 * rng.randn(*params[n].shape)
    x = rng.rand(B, *img)
    y = rng.randint(0, 5, size=B)
    o = od.DenseNetOracle(layers, params, state)
    loss, _, _, cache = o.forward(x, y, train=True)
    grads = o.backward(cache)
    tl, tg = torch_loss(layers, params, x, y)
    assert abs(loss - tl) <= 1e-12 * max(1.0, abs(tl))
    for n in params:
        np.testing.assert_allclose(grads[n], tg[n], rtol=1e-9, atol=1e-12, err_msg=n)


def test_arch_geometry_reference_config():
    # base_model.py:84-92 grid: depth 10, 3 blocks, growth 12, nb_filter 16
    layers = od.arch_layers(img_dim=(32, 32, 3), nb_classes=10)
    kinds = [ly["kind"] for ly in layers]
    assert kinds == ["conv0", "dense", "dense", "trans", "dense", "dense", "trans", "dense", "dense", "head"]
    assert [ly["cin"] for ly in layers] == [3, 16, 28, 40, 40, 52, 64, 64, 76, 88]
    assert [(ly["H"], ly["W"]) for ly in layers if ly["kind"] == "trans"] == [(32, 32), (16, 16)]
    assert layers[-1]["H"] == 8
    # ~23 MFLOP forward per sample
    assert 20e6 < od.flops_per_sample_fwd(layers) < 26e6


def test_bn_moving_stats_and_eval_mode():
    layers = od.arch_layers(img_dim=(8, 8, 3), nb_classes=4, depth=7, nb_dense_block=2, growth_rate=4, nb_filter=4)
    params, state = od.he_uniform_init(layers, seed=0)
    rng = np.random.RandomState(0)
    x = rng.rand(4, 8, 8, 3)
    y = rng.randint(0, 4, 4)
    o = od.DenseNetOracle(layers, params, state)
    _, _, _, c = o.forward(x, y, train=True)
    i = 1
    np.testing.assert_allclose(o.state[f"mm{i}"], 0.01 * c[i][1]["mean"])
    np.testing.assert_allclose(o.state[f"mv{i}"], 0.99 + 0.01 * c[i][1]["var"])
    s, correct = o.eval_batch(x, y)
    assert np.isfinite(s) and 0 <= correct <= 4


def test_torch_cpu_baseline_trajectory_matches_oracle():
    """oracle/densenet_torch.py (the timed CPU baseline) trains the same network:
    fp64 to 1e-10 of the oracle over 3 Adam steps, fp32 within 1e-3."""
    from oracle import densenet_torch as dt

    layers = od.arch_layers(img_dim=(12, 10, 3), nb_classes=5, depth=10, nb_dense_block=2, growth_rate=4,
                            nb_filter=6)
    params, state = od.he_uniform_init(layers, seed=2)
    rng = np.random.RandomState(4)
    x = rng.rand(4, 12, 10, 3)
    y = rng.randint(0, 5, size=4)
    o = od.DenseNetOracle(layers, params, state, lr=1e-2)
    n64 = dt.TorchDenseNet(layers, params, state, lr=1e-2, dtype=torch.float64)
    n32 = dt.TorchDenseNet(layers, params, state, lr=1e-2)
    for _ in range(3):
        ref = o.train_step(x, y)
        l64 = n64.train_step(torch.tensor(x), torch.tensor(y))
        l32 = n32.train_step(torch.tensor(x, dtype=torch.float32), torch.tensor(y))
        assert abs(l64 - ref) <= 1e-10 * abs(ref)
        assert abs(l32 - ref) <= 1e-3 * abs(ref)
    for i, ly in enumerate(layers):
        if ly["kind"] != "conv0":
            np.testing.assert_allclose(n64.S[f"mm{i}"].numpy(), o.state[f"mm{i}"], rtol=1e-9, atol=1e-12)
    s64, c64 = n64.eval_batch(torch.tensor(x), torch.tensor(y))
    s_ref, c_ref = o.eval_batch(x, y)
    assert abs(s64 - s_ref) <= 1e-9 * abs(s_ref) and c64 == c_ref
