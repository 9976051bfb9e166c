"""DenseNet population (csrc/densenet.hip through the C ABI) vs the float64
oracle (oracle/densenet.py, itself pinned to torch autograd in
test_oracle_densenet.py), on identical init, data order and learning rates.

Tolerances (f32 device vs f64 oracle): loss 1e-4 relative per step and the
north_star's 1e-3 relative over a multi-step trajectory; gradients per tensor
within 2e-3 of the tensor's max |g| (BN backward subtracts two sums of
B*W*C terms, so the f32 error scales with the tensor, not the element)."""
import numpy as np
import pytest
import torch

from oracle import densenet as od

pytestmark = pytest.mark.gpu


def _setup(img, classes, depth, blocks, growth, nbf, lrs, B, n_samples, seed=0):
    from mpi_opt_amd.densenet import DenseNetArch, DenseNetPopulation, he_uniform_init

    arch = DenseNetArch(img_dim=img, nb_classes=classes, depth=depth, nb_dense_block=blocks, growth_rate=growth,
                        nb_filter=nbf)
    layers = od.arch_layers(img_dim=img, nb_classes=classes, depth=depth, nb_dense_block=blocks,
                            growth_rate=growth, nb_filter=nbf)
    rng = np.random.RandomState(seed)
    init = []
    for i in range(len(lrs)):
        p, s = he_uniform_init(layers, 100 + i)
        for n in p:   # non-trivial BN affine
            if n[0] in "gb" and n != "bd":
                p[n] = (p[n] + 0.2 * rng.randn(*p[n].shape)).astype(np.float32)
        init.append((p, s))
    pop = DenseNetPopulation(arch, lrs, batch=B, init=init)
    x = rng.rand(n_samples, *img).astype(np.float32)
    y = rng.randint(0, classes, n_samples).astype(np.int32)
    order = np.stack([rng.permutation(n_samples).astype(np.int32) for _ in lrs])
    dev = torch.device("cuda")
    return pop, layers, init, x, y, order, torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev), \
        torch.from_numpy(order).to(dev)


def _oracle(layers, init_i, lr):
    p, s = init_i
    return od.DenseNetOracle(layers, {k: v.astype(np.float64) for k, v in p.items()},
                             {k: v.astype(np.float64) for k, v in s.items()}, lr=lr)


CASES = [
    # BASELINE config 5 geometry (CIFAR-10 shape, base_model.py grid)
    dict(img=(32, 32, 3), classes=10, depth=10, blocks=3, growth=12, nbf=16, B=6),
    # odd spatial sizes (floor-mode AvgPool), 2 blocks, ragged channel counts
    dict(img=(9, 11, 2), classes=5, depth=7, blocks=2, growth=5, nbf=7, B=5),
    # wide dense layers: the second has 9 x 90 = 810 weight-gradient rows (two 768-row
    # m-groups), growth 30 (two 16-column tiles)
    dict(img=(8, 8, 3), classes=4, depth=10, blocks=1, growth=30, nbf=60, B=4),
    # a pooled transition epilogue (10-row chunk) over an odd width: AvgPool2 drops column 8
    dict(img=(10, 9, 3), classes=3, depth=7, blocks=2, growth=8, nbf=12, B=4),
]


@pytest.mark.parametrize("case", CASES, ids=["cifar-d10", "odd-d7", "wide-d10", "pooled-odd-w"])
def test_forward_loss_and_gradients(case):
    lrs = [1e-3, 3e-4, 1e-2]
    pop, layers, init, x, y, order, xd, yd, od_ = _setup(case["img"], case["classes"], case["depth"], case["blocks"],
                                                         case["growth"], case["nbf"], lrs, case["B"], 40)
    B = case["B"]
    loss = pop.train_step(xd, yd, od_, 0).cpu().numpy()
    for i, lr in enumerate(lrs):
        o = _oracle(layers, init[i], lr)
        idx = order[i, :B]
        ol, _, _, cache = o.forward(x[idx], y[idx], train=True)
        grads = o.backward(cache)
        assert abs(loss[i] - ol) <= 1e-4 * abs(ol), (i, loss[i], ol)
        dg = pop.get_grads(i)
        for n, g in grads.items():
            dev = dg[n].astype(np.float64) + 2 * od.L2 * init[i][0][n].astype(np.float64)
            scale = np.abs(g).max() + 1e-12
            err = np.abs(dev - g).max() / scale
            assert err <= 2e-3, (i, n, err)
        st = pop.get_state(i)
        for n, v in o.state.items():
            np.testing.assert_allclose(st[n], v, rtol=1e-4, atol=1e-5, err_msg=n)


def test_training_trajectory_and_eval_within_1e3():
    case = CASES[0]
    lrs = [1e-3, 5e-3]
    B = 6
    steps = 4
    pop, layers, init, x, y, order, xd, yd, od_ = _setup(case["img"], case["classes"], case["depth"], case["blocks"],
                                                         case["growth"], case["nbf"], lrs, B, 40, seed=1)
    oracles = [_oracle(layers, init[i], lr) for i, lr in enumerate(lrs)]
    for s in range(steps):
        dl = pop.train_step(xd, yd, od_, s * B).cpu().numpy()
        for i, o in enumerate(oracles):
            idx = order[i, s * B:(s + 1) * B]
            ol = o.train_step(x[idx], y[idx])
            assert abs(dl[i] - ol) <= 1e-3 * abs(ol), (s, i, dl[i], ol)
    # inference-mode validation batch (BN moving averages)
    pop.eval_reset()
    pop.eval_step(xd, yd, od_, 30)
    vs = pop.val_loss_sum.cpu().numpy()
    vc = pop.val_correct.cpu().numpy()
    pen = pop.penalty().cpu().numpy()
    for i, o in enumerate(oracles):
        idx = order[i, 30:30 + B]
        s_, c_ = o.eval_batch(x[idx], y[idx])
        assert abs(vs[i] - s_) <= 1e-3 * abs(s_), (i, vs[i], s_)
        assert vc[i] == c_
        assert abs(pen[i] - o.l2_penalty()) <= 1e-4 * o.l2_penalty()


def test_member_isolation_bit_identical():
    """A member trains bit-identically alone or inside a population."""
    from mpi_opt_amd.densenet import DenseNetArch, DenseNetPopulation, he_uniform_init

    arch = DenseNetArch(img_dim=(16, 16, 3), nb_classes=10, depth=7, nb_dense_block=3, growth_rate=12, nb_filter=16)
    layers = od.arch_layers(img_dim=(16, 16, 3), nb_classes=10, depth=7, nb_dense_block=3, growth_rate=12,
                            nb_filter=16)
    init = [he_uniform_init(layers, 7 + i) for i in range(3)]
    rng = np.random.RandomState(5)
    x = torch.from_numpy(rng.rand(64, 16, 16, 3).astype(np.float32)).cuda()
    y = torch.from_numpy(rng.randint(0, 10, 64).astype(np.int32)).cuda()
    order = torch.from_numpy(np.stack([rng.permutation(64).astype(np.int32) for _ in range(3)])).cuda()
    full = DenseNetPopulation(arch, [1e-3, 2e-3, 4e-3], batch=8, init=init)
    solo = DenseNetPopulation(arch, [2e-3], batch=8, init=[init[1]])
    for s in range(3):
        full.train_step(x, y, order, s * 8)
        solo.train_step(x, y, order[1:2].contiguous(), s * 8)
    torch.cuda.synchronize()
    assert torch.equal(full.params[1], solo.params[0])
    assert torch.equal(full.state[1], solo.state[0])


def test_member_isolation_at_the_reference_batch():
    """At batch 100 the work splits (weight-gradient sample groups, BN batch
    slices) are sized for a nominal population: a member of a 24-member population
    and the same member alone take the same partial-sum orders, so the same bits
    (split by the actual population size, 24 members would use 2-sample groups and
    6 BN slices, one member 1-sample groups and 100 slices)."""
    from mpi_opt_amd.densenet import DenseNetArch, DenseNetPopulation, he_uniform_init

    arch = DenseNetArch(img_dim=(16, 16, 3), nb_classes=10, depth=7, nb_dense_block=3, growth_rate=12, nb_filter=16)
    layers = od.arch_layers(img_dim=(16, 16, 3), nb_classes=10, depth=7, nb_dense_block=3, growth_rate=12,
                            nb_filter=16)
    n, k, B = 24, 5, 100
    init = [he_uniform_init(layers, 11 + i) for i in range(n)]
    rng = np.random.RandomState(9)
    x = torch.from_numpy(rng.rand(2 * B, 16, 16, 3).astype(np.float32)).cuda()
    y = torch.from_numpy(rng.randint(0, 10, 2 * B).astype(np.int32)).cuda()
    order = torch.from_numpy(np.stack([rng.permutation(2 * B).astype(np.int32) for _ in range(n)])).cuda()
    lrs = [1e-3 * (1 + i % 4) for i in range(n)]
    full = DenseNetPopulation(arch, lrs, batch=B, init=init)
    solo = DenseNetPopulation(arch, [lrs[k]], batch=B, init=[init[k]])
    for s in range(2):
        full.train_step(x, y, order, s * B)
        solo.train_step(x, y, order[k:k + 1].contiguous(), s * B)
    torch.cuda.synchronize()
    assert torch.equal(full.params[k], solo.params[0])
    assert torch.equal(full.state[k], solo.state[0])


def test_fit_folds_reference_config_runs():
    from mpi_opt_amd.densenet import DenseNetArch, DenseNetPopulation, synthetic_cifar

    x, y = synthetic_cifar(n=400, seed=3)
    pop = DenseNetPopulation(DenseNetArch(), [1e-3] * 5, batch=20)
    h = pop.fit_folds(x, y, folds=list(range(5)), n_fold=5, epochs=2, record_train_loss=True)
    assert h["val_loss"].shape == (5, 2) and np.isfinite(h["val_loss"]).all()
    assert h["train_loss"].shape == (5, 2 * h["steps_per_epoch"])
    assert np.isfinite(h["train_loss"]).all()


def test_trial_evaluator_routes_densenet_specs():
    """BuilderFromFunction(test_densenet) -> TrialEvaluator trains DenseNet trials
    as one population and returns fold-mean validation losses (FOMs)."""
    from mpi_opt_amd.blocks import TrialEvaluator
    from mpi_opt_amd.densenet import synthetic_cifar
    from mpi_opt_amd.models import BuilderFromFunction, test_densenet
    from mpi_opt_amd.space import Real

    prov = BuilderFromFunction(lambda llr: test_densenet(nb_classes=10, img_dim=(16, 16, 3), depth=7,
                                                         lr=10.0 ** llr), [Real(-5.0, 1.0, name="llr")])
    x, y = synthetic_cifar(n=120, img_dim=(16, 16, 3), seed=1)
    ev = TrialEvaluator(prov, x, y, n_fold=2, epochs=1, batch=20)
    foms = ev.evaluate([[-3.0], [-2.0], [-4.0]])
    assert len(foms) == 3 and all(np.isfinite(foms))
    # the JSON is a Keras functional Model: its compiled lr is not part of to_json, so
    # every trial trains with the evaluator's lr; the trials differ by their init seeds
    assert all(ev.model_provider.builder(*p).spec(lr=ev.lr).lr == ev.lr for p in ([-3.0], [-2.0]))
    assert len(set(round(f, 6) for f in foms)) == 3


def test_side_stream_weight_gradients_bit_identical(monkeypatch):
    """The weight gradients on a second stream (default) vs one stream
    (MPO_DN_PLAN=streams=1): the same parameters and BN state, bit for bit,
    after 3 train steps (reference-grid architecture, 3 members)."""
    from mpi_opt_amd.densenet import DenseNetArch, DenseNetPopulation, he_uniform_init

    arch = DenseNetArch(img_dim=(32, 32, 3), nb_classes=10, depth=10, nb_dense_block=3, growth_rate=12, nb_filter=16)
    layers = od.arch_layers(img_dim=(32, 32, 3), nb_classes=10, depth=10, nb_dense_block=3, growth_rate=12,
                            nb_filter=16)
    init = [he_uniform_init(layers, 11 + i) for i in range(3)]
    rng = np.random.RandomState(6)
    x = torch.from_numpy(rng.rand(64, 32, 32, 3).astype(np.float32)).cuda()
    y = torch.from_numpy(rng.randint(0, 10, 64).astype(np.int32)).cuda()
    order = torch.from_numpy(np.stack([rng.permutation(64).astype(np.int32) for _ in range(3)])).cuda()
    out = []
    for plan in ("streams=1", "streams=2"):
        monkeypatch.setenv("MPO_DN_PLAN", plan)
        pop = DenseNetPopulation(arch, [1e-3, 2e-3, 4e-3], batch=16, init=init)
        for s in range(3):
            pop.train_step(x, y, order, s * 16)
        torch.cuda.synchronize()
        out.append((pop.params.clone(), pop.state.clone()))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


def test_streamed_1x1_conv_matches_the_staged_kernel(monkeypatch):
    """r05: the transitions' 1x1 convs (forward with BN + ELU and the AvgPool2
    epilogue, and their input gradient) run on dn_conv1x1_kernel, which streams
    each wave's 2 x 8 pixel patch from HBM without LDS staging and walks K in
    16-channel float4 blocks.  Only the order of the K sum differs from
    dn_conv_kernel (MPO_DN_PLAN=c1x1=0): one step's gradients agree to f32
    rounding, and the oracle tests above run on the streamed kernel."""
    case = CASES[0]
    grads = []
    for plan in ("", "c1x1=0"):
        if plan:
            monkeypatch.setenv("MPO_DN_PLAN", plan)
        else:
            monkeypatch.delenv("MPO_DN_PLAN", raising=False)
        pop, layers, init, x, y, order, xd, yd, od_ = _setup(case["img"], case["classes"], case["depth"],
                                                             case["blocks"], case["growth"], case["nbf"],
                                                             [1e-3, 3e-2], case["B"], 4 * case["B"], seed=5)
        pop.train_step(xd, yd, od_, 0)
        torch.cuda.synchronize()
        grads.append((pop.grads.clone(), pop.loss.clone()))
    (ga, la), (gb, lb) = grads
    assert float((ga - gb).abs().max()) <= 1e-5 * float(gb.abs().max())
    assert torch.allclose(la, lb, rtol=1e-5, atol=0)
