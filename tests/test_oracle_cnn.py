"""Pin the CNN oracle (oracle/cnn.py, hand-written numpy backward) against an
independent implementation: torch CPU autograd (fp64) of the same Keras-semantics
model (NHWC flatten, floor-mode max-pool, inverted dropout, clipped BCE on softmax).
Keras/TF/mpi_learn themselves are absent, so parity with the literal reference
is unpinned; this pins the restatement's arithmetic."""
import numpy as np
import pytest
import torch

from oracle import cnn as C


def init_params(F, k, p, dense, seed):
    rng = np.random.RandomState(seed)
    out = {}
    for name, shape in C.param_shapes(F, k, p, dense):
        if name.startswith("w"):
            if len(shape) == 4:
                fan_in, fan_out = shape[0] * shape[1] * shape[2], shape[0] * shape[1] * shape[3]
            else:
                fan_in, fan_out = shape
            lim = np.sqrt(6.0 / (fan_in + fan_out))
            out[name] = rng.uniform(-lim, lim, size=shape)
        else:
            out[name] = rng.uniform(-0.1, 0.1, size=shape)   # non-zero biases exercise the bias grads
    return out


def torch_loss(params, x, y, p, masks, rate):
    P = {n: torch.tensor(v, dtype=torch.float64, requires_grad=True) for n, v in params.items()}
    B = x.shape[0]
    t = torch.tensor(x.reshape(B, 28, 28, 1), dtype=torch.float64).permute(0, 3, 1, 2)
    w1 = P["w1"].permute(3, 2, 0, 1)
    w2 = P["w2"].permute(3, 2, 0, 1)
    a1 = torch.relu(torch.nn.functional.conv2d(t, w1) + P["b1"][None, :, None, None])
    a2 = torch.relu(torch.nn.functional.conv2d(a1, w2) + P["b2"][None, :, None, None])
    pool = torch.nn.functional.max_pool2d(a2, p)                       # floor mode
    flat = pool.permute(0, 2, 3, 1).reshape(B, -1)                     # NHWC flatten
    keep = 1.0 - rate
    pd = flat * torch.tensor(masks[0].reshape(flat.shape) / keep)
    h = torch.relu(pd @ P["w3"] + P["b3"])
    hd = h * torch.tensor(masks[1].reshape(h.shape) / keep)
    prob = torch.softmax(hd @ P["w4"] + P["b4"], dim=1)
    onehot = torch.nn.functional.one_hot(torch.tensor(y), 10).to(torch.float64)
    pc = torch.clamp(prob, 1e-7, 1 - 1e-7)
    loss = (-(onehot * torch.log(pc) + (1 - onehot) * torch.log(1 - pc))).mean(1).mean()
    loss.backward()
    return float(loss), {n: v.grad.numpy() for n, v in P.items()}


@pytest.mark.parametrize("F,k,p,dense", [(10, 2, 2, 50), (13, 5, 3, 64), (20, 10, 10, 200), (7, 3, 7, 33)])
def test_forward_and_gradients_match_torch_autograd(F, k, p, dense):
    B = 6
    rng = np.random.RandomState(1)
    x = rng.uniform(size=(B, 784))
    y = rng.randint(0, 10, size=B)
    params = init_params(F, k, p, dense, seed=F + k)
    o = C.TrialOracle(F, k, p, dense, params, dropout=0.25, seed=77)
    loss, _, _, cache = o.forward(x, y, step=3, train=True)
    grads = o.backward(cache)
    g = C.geometry(F, k, p, dense)
    m1 = C.dropout_keep(77, 3, 0, B * g["K1"], 0.25)
    m2 = C.dropout_keep(77, 3, 1, B * dense, 0.25)
    tl, tg = torch_loss(params, x, y, p, (m1, m2), 0.25)
    assert abs(loss - tl) < 1e-12 * abs(tl)
    for n in grads:
        np.testing.assert_allclose(grads[n], tg[n], rtol=1e-9, atol=1e-14, err_msg=n)


def test_adam_keras_form():
    params = init_params(10, 2, 2, 50, seed=0)
    o = C.TrialOracle(10, 2, 2, 50, params, lr=1e-3)
    g = {n: np.full_like(v, 0.5) for n, v in o.params.items()}
    w0 = o.params["w3"].copy()
    o.adam(g)
    # t=1: m = 0.05, v = 0.00025, lr_t = lr*sqrt(1-b2)/(1-b1)
    lr_t = 1e-3 * np.sqrt(1 - 0.999) / (1 - 0.9)
    np.testing.assert_allclose(o.params["w3"], w0 - lr_t * 0.05 / (np.sqrt(0.00025) + 1e-8), rtol=1e-14, atol=1e-16)


def test_dropout_hash_is_deterministic_and_unbiased():
    a = C.dropout_keep(5, 10, 0, 200000, 0.25)
    b = C.dropout_keep(5, 10, 0, 200000, 0.25)
    assert np.array_equal(a, b)
    assert abs(a.mean() - 0.75) < 0.005
    c = C.dropout_keep(5, 11, 0, 200000, 0.25)
    assert 0.5 < (a == c).mean() < 0.7      # independent streams per step
    assert C.dropout_keep(5, 10, 0, 100, 0.0).all()


def test_flop_formula():
    # SURVEY §8d formula at (F,k,p,dense) = (30,6,6,125)
    f = C.flops_per_sample_fwd(30, 6, 6, 125)
    assert f == 2 * 36 * 30 * 23 ** 2 + 2 * 36 * 900 * 18 ** 2 + 2 * 9 * 30 * 125 + 20 * 125
