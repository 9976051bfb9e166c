"""Long-trajectory parity cases shared by the fixture generator
(tests/golden/make_trajectory_golden.py, runs the fp64 oracles on the host) and
the GPU tests (tests/test_trajectories_gpu.py, run the device populations).

Everything a case needs -- data, init weights, fold orders, dropout seeds -- is a
function of numpy seeds, so both sides rebuild it identically.
"""
from __future__ import annotations

import numpy as np

BATCH = 100

# ---------------------------------------------------------------------------
# configs[2]: 64 ragged trials x 5 folds = 320 members on one GPU, per-trial
# widths / lr / dropout, 20 train steps; 8 sampled members checked
# ---------------------------------------------------------------------------
POP_TRIALS, POP_FOLDS, POP_SAMPLES, POP_STEPS = 64, 5, 2000, 20


def pop_trials(seed=13579):
    """(F, k, p, dense, lr, dropout) drawn like bench.py's sample_trials."""
    rng = np.random.RandomState(seed)
    out = []
    for _ in range(POP_TRIALS):
        F, p, k, dense = int(rng.randint(10, 51)), int(rng.randint(2, 11)), int(rng.randint(2, 11)), \
            int(rng.randint(50, 201))
        out.append((F, k, p, dense, float(10.0 ** rng.uniform(-4, -2)), float(rng.uniform(0.0, 0.5))))
    return out


def pop_members():
    """[(F, k, p, dense, lr, dropout, fold, dropout_seed, init_seed)] for all 320 members."""
    out = []
    for t, (F, k, p, d, lr, dr) in enumerate(pop_trials()):
        for f in range(POP_FOLDS):
            i = len(out)
            out.append((F, k, p, d, lr, dr, f, 5000 + i, 9000 + i))
    return out


def pop_sampled():
    """8 member indices: every NT bucket (F <= 16/32/48/64), small and large k,
    the smallest and largest lr and dropout of the population."""
    m = pop_members()
    picks = []

    def add(i):
        if i not in picks:
            picks.append(i)

    for lo, hi in ((10, 16), (17, 32), (33, 48), (49, 50)):
        add(next(i for i, mm in enumerate(m) if lo <= mm[0] <= hi))
    add(int(np.argmin([mm[4] for mm in m])))
    add(int(np.argmax([mm[4] for mm in m])))
    add(int(np.argmax([mm[5] for mm in m])))
    add(int(np.argmax([mm[1] for mm in m])))
    i = len(m) - 1
    while len(picks) < 8:
        add(i)
        i -= 7
    return picks[:8]


def pop_data():
    rng = np.random.RandomState(21)
    x = rng.uniform(size=(POP_SAMPLES, 784)).astype(np.float32)
    y = rng.randint(0, 10, size=POP_SAMPLES).astype(np.int32)
    return x, y


# ---------------------------------------------------------------------------
# one full 5-fold fold-epoch (480 steps of 100 on 48 000 samples) + validation
# over the fold's 12 000 samples, 2 members
# ---------------------------------------------------------------------------
EPOCH_SAMPLES, EPOCH_FOLDS = 60000, 5
EPOCH_MEMBERS = [  # (F, k, p, dense, lr, dropout, fold, dropout_seed, init_seed)
    (24, 3, 2, 100, 1e-3, 0.25, 1, 71, 81),
    (45, 6, 3, 180, 5e-4, 0.25, 4, 72, 82),
]


def epoch_data():
    rng = np.random.RandomState(22)
    x = rng.uniform(size=(EPOCH_SAMPLES, 784)).astype(np.float32)
    y = rng.randint(0, 10, size=EPOCH_SAMPLES).astype(np.int32)
    return x, y


# ---------------------------------------------------------------------------
# DenseNet, BASELINE configs[4] geometry at batch 100, 20 steps
# ---------------------------------------------------------------------------
DN_LRS, DN_SAMPLES, DN_STEPS = [1e-3, 1e-2], 2000, 20


def dn_data():
    rng = np.random.RandomState(23)
    x = rng.rand(DN_SAMPLES, 32, 32, 3).astype(np.float32)
    y = rng.randint(0, 10, DN_SAMPLES).astype(np.int32)
    order = np.stack([rng.permutation(DN_SAMPLES).astype(np.int32) for _ in DN_LRS])
    return x, y, order


# ---------------------------------------------------------------------------
# DenseNet, BASELINE configs[4]: a 32-member population (the bench's lr draw
# 10**U(-5, 1)), 4 sampled members checked for 10 steps
# ---------------------------------------------------------------------------
DN32_LRS = 10.0 ** np.random.RandomState(2024).uniform(-5, 1, size=32)
DN32_STEPS = 10
DN32_PICKS = [int(np.argmin(np.abs(np.log10(DN32_LRS) - np.log10(t)))) for t in (1e-5, 2e-3, 4e-2, 0.4)]


def dn32_order():
    rng = np.random.RandomState(24)
    return np.stack([rng.permutation(DN_SAMPLES).astype(np.int32) for _ in DN32_LRS])


def glorot_init(F, k, p, dense, seed):
    """Same draw as mpi_opt_amd.population.glorot_uniform_init (Keras order)."""
    H2 = 28 - 2 * (k - 1)
    K1 = (H2 // p) ** 2 * F
    shapes = [("w1", (k, k, 1, F)), ("b1", (F,)), ("w2", (k, k, F, F)), ("b2", (F,)),
              ("w3", (K1, dense)), ("b3", (dense,)), ("w4", (dense, 10)), ("b4", (10,))]
    rng = np.random.RandomState(seed)
    out = {}
    for name, shape in shapes:
        if name.startswith("w"):
            if len(shape) == 4:
                fan_in, fan_out = shape[0] * shape[1] * shape[2], shape[0] * shape[1] * shape[3]
            else:
                fan_in, fan_out = shape
            lim = np.sqrt(6.0 / (fan_in + fan_out))
            out[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
        else:
            out[name] = np.zeros(shape, dtype=np.float32)
    return out
