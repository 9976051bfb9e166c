"""Device GP refit (``mpo_gp_lml_grad`` + the lockstep L-BFGS-B driver) against
scikit-learn's own outputs (golden ``gp_lml.npz``, made by
``tests/golden/make_lml_golden.py``).  n > 48 runs the split block sweep (one
many-workgroup step launch per 32-wide pivot block); n = 256 and 500 are the sizes a
256-trial search reaches (real points plus the cl_min lies of a batch ask);
MPO_FIT_KERNEL=panel / split re-checks each kernel outside its range."""
import os
import time

import numpy as np
import pytest
import torch

from oracle import gp_ei as O
from tests.conftest import ROOT

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(ROOT, "tests", "golden", "gp_lml.npz"))
CASES = ["n200_d10", "n12_d5", "n57_d3", "n230_d4", "n130_d6", "n256_d10", "n500_d10"]


SWEEP_MIN_N = 48      # csrc/gp_fit.hip kSplitMinN: above it the split block sweep


def _sweep(n):
    k = os.environ.get("MPO_FIT_KERNEL")
    return k == "split" or (k != "panel" and SWEEP_MIN_N < n)


def _rel_tol(X, theta):
    """fp64 rounding of the LML pieces grows with cond(K); sklearn's LAPACK
    solves and the device's explicit L^-1 round differently by up to ~cond*eps.
    The block-sweep kernels (n > 192) invert K by Gauss-Jordan sweeps instead of
    a Cholesky factor: the same ~cond*eps order with a 20x larger constant
    (measured up to 525 cond*eps, n = 130 forced through the split sweep)."""
    n, d = X.shape
    c = 1000.0 if _sweep(n) else 50.0
    amp, ls, noise = np.exp(theta[0]), np.exp(theta[1:d + 1]), np.exp(theta[d + 1])
    M = O.matern52(X, X, ls, 1.0)
    np.fill_diagonal(M, 1.0)
    K = amp * M + (noise + 1e-10) * np.eye(n)
    return max(1e-9, c * np.finfo(float).eps * np.linalg.cond(K))


def _lml(name):
    from mpi_opt_amd.gp_fit import DeviceLML, normalize_targets

    X, y = G[name + "_X"], G[name + "_y"]
    return DeviceLML(X, normalize_targets(y)[0], device="cuda:0"), X


@pytest.mark.parametrize("name", CASES)
def test_lml_and_gradient_match_sklearn(name):
    dev, X = _lml(name)
    T = G[name + "_theta"]
    lml, grad, info = dev.evaluate(T)
    assert np.all(info == 0)
    for b in range(len(T)):
        tol = _rel_tol(X, T[b])
        ref_l, ref_g = G[name + "_lml"][b], G[name + "_grad"][b]
        assert abs(lml[b] - ref_l) <= tol * max(1.0, abs(ref_l)), (b, lml[b], ref_l, tol)
        err = np.max(np.abs(grad[b] - ref_g)) / max(1.0, np.max(np.abs(ref_g)))
        assert err <= tol, (b, err, tol)


@pytest.mark.parametrize("name", ["n200_d10", "n230_d4", "n500_d10"])
def test_batching_does_not_change_results(name):
    dev, _ = _lml(name)
    T = G[name + "_theta"]
    lml, grad, _ = dev.evaluate(T)
    for b in range(len(T)):
        l1, g1, _ = dev.evaluate(T[b:b + 1])
        assert l1[0] == lml[b] and np.array_equal(g1[0], grad[b])


@pytest.mark.parametrize("name", ["n256_d10", "n500_d10"])
def test_full_batch_step_tiles_per_wave_keep_bits(name):
    """40 thetas in one launch set: the step kernel's waves take several tiles each
    (csrc/gp_fit.hip kStepWgTarget), one theta alone takes one tile per wave -- the
    same bits either way."""
    from mpi_opt_amd.gp_fit import theta_bounds

    dev, X = _lml(name)
    b = theta_bounds(X.shape[1])
    T = np.random.RandomState(7).uniform(b[:, 0], b[:, 1], size=(40, X.shape[1] + 2))
    lml, grad, info = dev.evaluate(T)
    for i in range(len(T)):
        l1, g1, i1 = dev.evaluate(T[i:i + 1])
        assert i1[0] == info[i]
        assert (l1[0] == lml[i] or (np.isnan(l1[0]) and np.isnan(lml[i]))) and np.array_equal(g1[0], grad[i]), i


@pytest.mark.parametrize("name,kernel", [("n200_d10", "panel"), ("n130_d6", "panel"), ("n57_d3", "split")])
def test_other_kernel_still_matches_sklearn(name, kernel, monkeypatch):
    """Each LML kernel outside its default range: the Cholesky kernel at n <= 200,
    the block sweep at small n (one pivot block with identity padding)."""
    monkeypatch.setenv("MPO_FIT_KERNEL", kernel)
    test_lml_and_gradient_match_sklearn(name)


@pytest.mark.parametrize("name", ["n12_d5"])
def test_split_sweep_at_small_n_matches_sklearn(name, monkeypatch):
    monkeypatch.setenv("MPO_FIT_KERNEL", "split")
    test_lml_and_gradient_match_sklearn(name)


@pytest.mark.parametrize("kernel", ["split"])
def test_non_finite_theta_reports_failure_in_sweeps(kernel, monkeypatch):
    monkeypatch.setenv("MPO_FIT_KERNEL", kernel)
    dev, _ = _lml("n230_d4")
    T = G["n230_d4_theta"][:2].copy()
    T[1, 0] = np.nan
    lml, grad, info = dev.evaluate(T)
    assert info[0] == 0 and info[1] >= 1
    assert lml[1] == -np.inf and np.all(grad[1] == 0.0)
    assert np.isfinite(lml[0])


def test_non_finite_theta_reports_cholesky_failure():
    dev, _ = _lml("n57_d3")
    T = G["n57_d3_theta"][:2].copy()
    T[1, 0] = np.nan
    lml, grad, info = dev.evaluate(T)
    assert info[0] == 0 and info[1] == 1
    assert lml[1] == -np.inf and np.all(grad[1] == 0.0)
    assert np.isfinite(lml[0])


@pytest.mark.parametrize("driver", ["native", "scipy"])
@pytest.mark.parametrize("name", CASES)
def test_device_fit_matches_sklearn_fit(name, driver):
    """Both L-BFGS-B drivers on the device objective: libmpo.so's host L-BFGS-B
    (mpo_gp_fit_lml_host) and scipy's setulb driven from Python."""
    from mpi_opt_amd.gp_fit import fit_lml

    X, y = G[name + "_X"], G[name + "_y"]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    (amp, ls, noise), det = fit_lml(X, y, random_state=int(G[name + "_seed"]), device="cuda:0",
                                    return_details=True, driver=driver)
    dt = time.perf_counter() - t0
    theta = np.log(np.r_[amp, ls, noise])
    ref = G[name + "_fit_theta"]
    print(f"{name} ({driver}): device fit {dt * 1e3:.1f} ms, {det['launches']} launches, lml {det['lml']:.9f}")
    # the LML at the optimum agrees tightly; theta within the optimiser's resolution
    assert abs(det["lml"] - float(G[name + "_fit_lml"])) <= 1e-7 * abs(float(G[name + "_fit_lml"]))
    assert np.max(np.abs(theta - ref)) <= 1e-3, (theta, ref)


def _batcher_stats():
    import ctypes

    from mpi_opt_amd import _lib

    la, ro = ctypes.c_int64(), ctypes.c_int64()
    _lib.check(_lib.lib().mpo_gp_lml_batcher_stats(_lib.lml_batcher(0), ctypes.byref(la), ctypes.byref(ro)))
    return la.value, ro.value


def test_concurrent_fits_share_launches_with_identical_results():
    """Refits on several threads at once (the cl_min chains) go through the
    device's batcher: rounds of different problems (n = 60 ... 201, d = 5 and 3:
    one launch set per d) launch together, and every fit's optima, values and
    counts equal its lone run on the plain per-round path (no batcher).  The
    threads start together (barrier), and fewer launch sets than rounds shows
    that rounds were actually grouped."""
    import threading

    from mpi_opt_amd.gp_fit import DeviceLML, normalize_targets, theta_bounds

    probs, bounds = [], []
    for n, seed, d in [(60, 1, 5), (96, 2, 5), (150, 3, 3), (201, 4, 5), (96, 5, 3), (75, 6, 5)]:
        X, y = O.synthetic_problem(n, d, seed=seed)
        probs.append((X, normalize_targets(y)[0]))
        bounds.append(theta_bounds(d))
    rng = np.random.RandomState(0)
    starts = [np.array([np.zeros(len(b))] + [rng.uniform(b[:, 0], b[:, 1]) for _ in range(2)]) for b in bounds]
    seq = [DeviceLML(X, yn, device="cuda:0").fit(st, b, batcher=False)
           for (X, yn), st, b in zip(probs, starts, bounds)]
    l0, r0 = _batcher_stats()
    out = [None] * len(probs)
    errors = []
    go = threading.Barrier(len(probs))

    def run(i):
        try:
            torch.cuda.set_device(0)
            with torch.cuda.stream(torch.cuda.Stream()):
                lml = DeviceLML(*probs[i], device="cuda:0")
                go.wait()
                out[i] = lml.fit(starts[i], bounds[i])
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    ths = [threading.Thread(target=run, args=(i,)) for i in range(len(probs))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors
    l1, r1 = _batcher_stats()
    print(f"{r1 - r0} rounds in {l1 - l0} grouped launch sets")
    for (a, ra), (c, rc) in zip(seq, out):
        assert ra == rc
        for (x1, f1), (x2, f2) in zip(a, c):
            assert np.array_equal(x1, x2) and f1 == f2
    assert r1 - r0 == sum(r for _, r in seq) and l1 - l0 < r1 - r0


def test_fused_split_sweep_reports_failure():
    dev, _ = _lml("n230_d4")
    T = G["n230_d4_theta"][:3].copy()
    T[1, 0] = np.nan
    lml, grad, info = dev.evaluate(T)
    assert info[0] == 0 and info[1] >= 1 and info[2] == 0
    assert lml[1] == -np.inf and np.all(grad[1] == 0.0)
    l2, g2, _ = dev.evaluate(T[2:3])
    assert l2[0] == lml[2] and np.array_equal(g2[0], grad[2])


@pytest.mark.parametrize("name", ["n130_d6", "n500_d10"])
def test_repeated_host_staged_calls_are_bit_identical(name):
    """The host-staged call (theta and the output rows in pinned host memory, the
    arrival counter of the last-workgroup sum re-armed per call): repeated calls
    give the same bits, and a failed theta still reports."""
    dev, _ = _lml(name)
    T = G[name + "_theta"]
    l0, g0, i0 = dev.evaluate(T)
    for _ in range(3):
        l1, g1, i1 = dev.evaluate(T)
        assert np.array_equal(i0, i1) and np.array_equal(l0, l1) and np.array_equal(g0, g1)
    T2 = T[:2].copy()
    T2[1, 0] = np.nan
    l2, g2, i2 = dev.evaluate(T2)
    assert i2[0] == 0 and i2[1] >= 1 and l2[1] == -np.inf and np.all(g2[1] == 0.0) and l2[0] == l0[0]


def test_lookahead_sweep_and_tile_build_keep_the_bits(tmp_path):
    """r06: the look-ahead pivot sweep (MPO_FIT_LOOKAHEAD) and the K build as 16x16
    tiles (MPO_FIT_BUILD) change the schedule, never an operation: the LML, gradient
    and status of 5 problems x 6 thetas plus 40-theta groups (n = 57 ... 500, the
    tiles-per-wave path included) are bit-identical to the r05 schedule.  The switches
    are read once per process, so each variant runs in its own (sequential) process."""
    import subprocess
    import sys

    probe = os.path.join(ROOT, "scripts", "lml_bits_probe.py")
    ref = str(tmp_path / "r05_schedule.npz")
    env0 = dict(os.environ, MPO_FIT_LOOKAHEAD="0", MPO_FIT_BUILD="rows")
    subprocess.run([sys.executable, probe, ref], env=env0, check=True, timeout=240)
    for name, extra in (("lookahead", {"MPO_FIT_BUILD": "rows"}), ("tiles", {"MPO_FIT_LOOKAHEAD": "0"}), ("both", {})):
        env = {k: v for k, v in os.environ.items() if k not in ("MPO_FIT_LOOKAHEAD", "MPO_FIT_BUILD")}
        env.update(extra)
        out = subprocess.run([sys.executable, probe, str(tmp_path / f"{name}.npz"), ref], env=env, check=True,
                             timeout=240, capture_output=True, text=True).stdout
        assert "bit-identical: True" in out, (name, out)
