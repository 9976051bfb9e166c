"""GPU parity of the population training engine (csrc/cnn.hip) against the fp64
numpy oracle (oracle/cnn.py) on identical seeded init weights, data order and
dropout masks.  Bar (BASELINE.json north_star): per-step training loss within
1e-3 relative.  Gradients are additionally checked tensor by tensor."""
import numpy as np
import pytest
import torch

from oracle import cnn as C

pytestmark = pytest.mark.gpu

# (F, k, p, dense, lr, dropout, fold): extremes of the option3 mnist space,
# every NT bucket (F <= 16, 32, 48, 64) and s = 1 pooling
MEMBERS = [
    (10, 2, 2, 50, 1e-3, 0.25, 0),
    (50, 10, 10, 200, 1e-3, 0.25, 1),
    (33, 5, 3, 77, 2e-3, 0.25, 2),
    (17, 3, 7, 120, 1e-3, 0.1, 3),
    (50, 2, 2, 200, 1e-3, 0.25, 4),
    (16, 7, 4, 64, 3e-3, 0.5, 0),
]
N_SAMPLES, N_FOLD, BATCH = 500, 5, 100

# ((F, k, p, dense, lr, dropout, fold), loss, optimizer): the mpi_learn --loss /
# --optimizer choices beside the reference's binary_crossentropy + adam
OPTION_MEMBERS = [
    ((12, 3, 2, 64, 1e-3, 0.25, 0), "categorical_crossentropy", "adam"),
    ((20, 5, 3, 80, 5e-2, 0.1, 1), "binary_crossentropy", "sgd"),
    ((33, 4, 2, 100, 5e-2, 0.25, 2), "categorical_crossentropy", "sgd"),
    ((17, 2, 4, 50, 2e-3, 0.5, 3), "binary_crossentropy", "adam"),
]


def dataset(seed=0):
    rng = np.random.RandomState(seed)
    x = rng.uniform(size=(N_SAMPLES, 784)).astype(np.float32)
    y = rng.randint(0, 10, size=N_SAMPLES).astype(np.int32)
    return x, y


def make_engine(members=MEMBERS, first=0):
    from mpi_opt_amd.population import PopulationEngine, TrialSpec, glorot_uniform_init

    specs = [TrialSpec(F, k, p, d, lr, dr, seed=1000 + first + i) for i, (F, k, p, d, lr, dr, _) in enumerate(members)]
    init = [glorot_uniform_init(s, 7 + first + i) for i, s in enumerate(specs)]
    eng = PopulationEngine(specs, batch=BATCH, init=init)
    return eng, specs, init


def oracle_for(spec, init):
    return C.TrialOracle(spec.nb_filters, spec.kernel_size, spec.pool_size, spec.dense,
                         {n: v.astype(np.float64) for n, v in init.items()}, lr=spec.lr,
                         dropout=spec.dropout, seed=spec.seed)


def orders(members, x):
    from mpi_opt_amd.population import kfold_split

    tr, va = [], []
    for m in members:
        t, v = kfold_split(x.shape[0], N_FOLD, m[-1])
        tr.append(t)
        va.append(v)
    return np.stack(tr), np.stack(va)


def test_eval_forward_matches_oracle():
    x, y = dataset()
    eng, specs, init = make_engine()
    tr, va = orders(MEMBERS, x)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    ova = torch.from_numpy(va).cuda()
    eng.eval_reset()
    eng.eval_step(xd, yd, ova, 0)
    got = eng.val_loss_sum.cpu().numpy() / BATCH
    for i, s in enumerate(specs):
        ref = oracle_for(s, init[i]).eval_loss(x[va[i]], y[va[i]])
        assert abs(got[i] - ref) <= 1e-5 * abs(ref), (i, got[i], ref)


def device_decisions(eng, i, spec):
    """The device forward's discrete choices (argmax, ReLU gates) for member i."""
    g = spec.geometry()
    F, D = spec.nb_filters, spec.dense
    am = eng.argmax_table(i).reshape(BATCH, g["s"], g["s"], F).astype(np.int64)
    return {"arg": am,
            "a1_pos": eng.activation(i, "a1", (BATCH, g["H1"], g["H1"], F)) > 0,
            "a2_pos": eng.activation(i, "a2", (BATCH, g["H2"], g["H2"], F)) > 0,
            "h_pos": eng.activation(i, "h", (BATCH, D)) > 0}


def test_one_step_gradients_match_oracle():
    x, y = dataset(1)
    eng, specs, init = make_engine()
    tr, va = orders(MEMBERS, x)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    otr = torch.from_numpy(tr).cuda()
    loss = eng.train_step(xd, yd, otr, 0).cpu().numpy()
    grads = eng.grads.cpu().numpy()
    report = []
    for i, s in enumerate(specs):
        o = oracle_for(s, init[i])
        ref_loss, _, _, cache = o.forward(x[tr[i][:BATCH]], y[tr[i][:BATCH]], step=0, train=True)
        g, absg = o.backward(cache, abs_terms=True, decisions=device_decisions(eng, i, s))
        assert abs(loss[i] - ref_loss) <= 1e-5 * abs(ref_loss), (i, loss[i], ref_loss)
        for j, (name, (off, shape)) in enumerate(eng._slices(i).items()):
            cnt = int(np.prod(shape))
            gd = grads[off:off + cnt].reshape(shape)
            # f32 bound: error of an n-term f32 reduction of already-f32-rounded
            # terms is O(1e-6) of the sum of |terms|, plus 1e-4 of the tensor scale
            err = np.abs(gd - g[name])
            bound = 1e-4 * np.abs(g[name]).max() + 2e-5 * absg[name]
            report.append((i, name, float((err / (np.abs(g[name]).max() + 1e-30)).max()),
                           float((err / (absg[name] + 1e-30)).max()), bool(np.all(err <= bound))))
    for r in report:
        print("member %d %-3s err/max %.2e err/sum|terms| %.2e ok=%s" % r)
    assert all(r[-1] for r in report)


@pytest.mark.parametrize("epochs", [2])
def test_multistep_losses_within_1e3(epochs):
    x, y = dataset(2)
    eng, specs, init = make_engine()
    tr, va = orders(MEMBERS, x)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    hist = eng.fit_folds(xd, yd, [m[-1] for m in MEMBERS], N_FOLD, epochs, record_train_loss=True)
    steps = hist["steps_per_epoch"]
    for i, s in enumerate(specs):
        o = oracle_for(s, init[i])
        ref_tl, ref_vl = [], []
        step = 0
        for ep in range(epochs):
            for st in range(steps):
                rows = tr[i][st * BATCH:(st + 1) * BATCH]
                ref_tl.append(o.train_step(x[rows], y[rows], step))
                step += 1
            ref_vl.append(o.eval_loss(x[va[i]], y[va[i]]))
        rel = np.abs(hist["train_loss"][i] - np.array(ref_tl)) / np.abs(ref_tl)
        assert rel.max() < 1e-3, (i, rel)
        relv = np.abs(hist["val_loss"][i] - np.array(ref_vl)) / np.abs(ref_vl)
        assert relv.max() < 1e-3, (i, relv)


def test_kfold_gather_kernel():
    from mpi_opt_amd.population import kfold_gather

    x, _ = dataset(3)
    xd = torch.from_numpy(x).cuda()
    idx = np.random.RandomState(0).permutation(N_SAMPLES)[:123].astype(np.int32)
    out = kfold_gather(xd, torch.from_numpy(idx).cuda())
    np.testing.assert_array_equal(out.cpu().numpy(), x[idx])


def test_population_isolation():
    """A member's trajectory does not depend on who else is in the population."""
    x, y = dataset(4)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    eng_all, specs, init = make_engine()
    tr, _ = orders(MEMBERS, x)
    eng_one, _, _ = make_engine(MEMBERS[2:3], first=2)
    for st in range(3):
        la = eng_all.train_step(xd, yd, torch.from_numpy(tr).cuda(), st * BATCH).cpu().numpy()
        lo = eng_one.train_step(xd, yd, torch.from_numpy(tr[2:3]).cuda(), st * BATCH).cpu().numpy()
        assert la[2] == lo[0]


def test_loss_and_optimizer_options_match_oracle():
    """Members with categorical_crossentropy and/or SGD (MpoCnnSpec.options)
    train in one population beside the reference's BCE + Adam: first-step
    gradients per tensor and 2 epochs of per-step train / per-epoch validation
    losses against the oracle's TrialOracle(loss=..., optimizer=...), 1e-3."""
    from mpi_opt_amd.population import PopulationEngine, TrialSpec, glorot_uniform_init

    members = [m for m, _, _ in OPTION_MEMBERS]
    specs = [TrialSpec(F, k, p, d, lr, dr, seed=2000 + i, loss=lo, optimizer=op)
             for i, ((F, k, p, d, lr, dr, _), lo, op) in enumerate(OPTION_MEMBERS)]
    init = [glorot_uniform_init(s, 40 + i) for i, s in enumerate(specs)]

    def oracle(i):
        s = specs[i]
        return C.TrialOracle(s.nb_filters, s.kernel_size, s.pool_size, s.dense,
                             {n: v.astype(np.float64) for n, v in init[i].items()}, lr=s.lr, dropout=s.dropout,
                             seed=s.seed, loss=s.loss, optimizer=s.optimizer)

    x, y = dataset(4)
    tr, va = orders(members, x)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    eng = PopulationEngine(specs, batch=BATCH, init=init)
    loss = eng.train_step(xd, yd, torch.from_numpy(tr).cuda(), 0).cpu().numpy()
    grads = eng.grads.cpu().numpy()
    for i, s in enumerate(specs):
        o = oracle(i)
        ref_loss, _, _, cache = o.forward(x[tr[i][:BATCH]], y[tr[i][:BATCH]], step=0, train=True)
        g, absg = o.backward(cache, abs_terms=True, decisions=device_decisions(eng, i, s))
        assert abs(loss[i] - ref_loss) <= 1e-5 * abs(ref_loss), (i, loss[i], ref_loss)
        for name, (off, shape) in eng._slices(i).items():
            gd = grads[off:off + int(np.prod(shape))].reshape(shape)
            bound = 1e-4 * np.abs(g[name]).max() + 2e-5 * absg[name]
            assert np.all(np.abs(gd - g[name]) <= bound), (i, s.loss, name)
    eng = PopulationEngine(specs, batch=BATCH, init=init)
    hist = eng.fit_folds(xd, yd, [m[-1] for m in members], N_FOLD, 2, record_train_loss=True)
    steps = hist["steps_per_epoch"]
    for i in range(len(specs)):
        o = oracle(i)
        ref_tl, ref_vl, step = [], [], 0
        for ep in range(2):
            for st in range(steps):
                rows = tr[i][st * BATCH:(st + 1) * BATCH]
                ref_tl.append(o.train_step(x[rows], y[rows], step))
                step += 1
            ref_vl.append(o.eval_loss(x[va[i]], y[va[i]]))
        assert (np.abs(hist["train_loss"][i] - ref_tl) / np.abs(ref_tl)).max() < 1e-3, (i, specs[i].loss)
        assert (np.abs(hist["val_loss"][i] - ref_vl) / np.abs(ref_vl)).max() < 1e-3, (i, specs[i].loss)


def test_unsupported_options_are_refused():
    from mpi_opt_amd import _lib
    from mpi_opt_amd.population import PopulationEngine, TrialSpec

    with pytest.raises(ValueError):
        PopulationEngine([TrialSpec(10, 2, 2, 50, loss="mse")], batch=BATCH)
    import ctypes

    arr = (_lib.MpoCnnSpec * 1)()
    arr[0] = _lib.MpoCnnSpec(10, 2, 2, 50, 1e-3, 0.25, 1, 0x7)          # no such loss code
    h = ctypes.c_void_p()
    assert _lib.lib().mpo_pop_create(arr, 1, BATCH, ctypes.byref(h)) != 0
    assert "options" in _lib.lib().mpo_last_error().decode()


def test_side_stream_schedule_is_bit_identical(monkeypatch):
    """MPO_POP_PLAN streams=3 (default: conv2 forward buckets over two streams, the
    weight gradients beside the input gradients, the input-gradient buckets over a
    third), streams=2 and streams=1 (one stream): the same parameters, bit for bit,
    after 3 train steps of the mixed population."""
    x, y = dataset(5)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    tr, _ = orders(MEMBERS, x)
    otr = torch.from_numpy(tr).cuda()
    out = []
    for streams in ("1", "2", "3"):
        monkeypatch.setenv("MPO_POP_PLAN", f"streams={streams}")
        eng, _, _ = make_engine()
        losses = [eng.train_step(xd, yd, otr, st * BATCH).cpu().numpy().copy() for st in range(3)]
        torch.cuda.synchronize()
        out.append((np.stack(losses), eng.params.cpu().numpy().copy()))
    for k in (1, 2):
        np.testing.assert_array_equal(out[0][0], out[k][0])
        np.testing.assert_array_equal(out[0][1], out[k][1])


def test_input_gradient_formulations_are_bit_identical(monkeypatch):
    """The conv2 input gradient as the halo-skipping gather kernel (MPO_POP_PLAN
    dgfwd=0) and as the forward conv over a zero-bordered dz2 (dgfwd=13: every k;
    the default takes it for k <= 4): every MFMA step multiplies the same operands,
    so losses and parameters agree bit for bit after 3 train steps, for k = 2..10
    and F both a multiple of 16 and not."""
    members = MEMBERS + [(32, 4, 2, 60, 1e-3, 0.25, 1), (21, 6, 2, 70, 1e-3, 0.25, 2), (48, 8, 3, 90, 1e-3, 0.25, 3),
                         (13, 9, 2, 40, 1e-3, 0.25, 4)]
    x, y = dataset(8)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    tr, _ = orders(members, x)
    otr = torch.from_numpy(tr).cuda()
    out = []
    for knob in ("dgfwd=0", "dgfwd=13"):
        monkeypatch.setenv("MPO_POP_PLAN", knob)
        eng, _, _ = make_engine(members)
        losses = [eng.train_step(xd, yd, otr, st * BATCH).cpu().numpy().copy() for st in range(3)]
        torch.cuda.synchronize()
        out.append((np.stack(losses), eng.params.cpu().numpy().copy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


def test_engines_sharing_side_streams_are_bit_identical():
    """Population engines of one process share the pooled side streams
    (mpo::pooled_side_stream): two engines alive and stepped alternately give the
    bits of one engine stepped alone."""
    x, y = dataset(6)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    tr, _ = orders(MEMBERS, x)
    otr = torch.from_numpy(tr).cuda()
    alone, _, _ = make_engine()
    ref = [alone.train_step(xd, yd, otr, st * BATCH).cpu().numpy().copy() for st in range(3)]
    ref_p = alone.params.cpu().numpy().copy()
    del alone
    a, _, _ = make_engine()
    b, _, _ = make_engine()
    for st in range(3):
        la = a.train_step(xd, yd, otr, st * BATCH).cpu().numpy()
        lb = b.train_step(xd, yd, otr, st * BATCH).cpu().numpy()
        np.testing.assert_array_equal(la, ref[st])
        np.testing.assert_array_equal(lb, ref[st])
    np.testing.assert_array_equal(a.params.cpu().numpy(), ref_p)
    np.testing.assert_array_equal(b.params.cpu().numpy(), ref_p)


def test_engines_on_two_threads_and_streams_keep_their_bits():
    """The ABI is thread-safe across streams (include/mpo.h): two engines stepped at
    once from two threads, each on its own torch stream, get side streams pooled for
    their own caller stream (mpo::pooled_side_stream keyed by caller stream, r06),
    finish without waiting on each other, and keep the bits of an engine stepped
    alone."""
    import threading

    x, y = dataset(6)
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    tr, _ = orders(MEMBERS, x)
    otr = torch.from_numpy(tr).cuda()
    alone, _, _ = make_engine()
    ref = [alone.train_step(xd, yd, otr, st * BATCH).cpu().numpy().copy() for st in range(4)]
    ref_p = alone.params.cpu().numpy().copy()
    del alone
    engines = [make_engine()[0] for _ in range(2)]
    torch.cuda.synchronize()
    losses = [[], []]
    errors = []
    go = threading.Barrier(2)

    def run(i):
        try:
            torch.cuda.set_device(0)
            st_ = torch.cuda.Stream()
            with torch.cuda.stream(st_):
                go.wait()
                for st in range(4):
                    losses[i].append(engines[i].train_step(xd, yd, otr, st * BATCH).clone())
            st_.synchronize()
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    ths = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ths), "engines on two streams deadlocked"
    assert not errors, errors
    for i in range(2):
        for st in range(4):
            np.testing.assert_array_equal(losses[i][st].cpu().numpy(), ref[st])
        np.testing.assert_array_equal(engines[i].params.cpu().numpy(), ref_p)
