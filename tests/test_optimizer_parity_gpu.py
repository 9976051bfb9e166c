"""G2 parity: the device ``Optimizer``'s ask/tell sequence against the CPU
restatement of skopt's loop (``oracle/skopt_optimizer.py``: sklearn's own GP fit,
skopt's einsum posterior, scipy L-BFGS-B polish, gp_hedge gains / softmax /
multinomial pick, cl_min lies through ``copy()``).

Reference: ``skopt.Optimizer(dimensions, random_state=13579)``
(/root/reference/coordinator.py:33), ``tell(X, Y)`` (:69), ``ask(num_iterations)``
(:49).  Both sides draw from the same ``RandomState`` stream; the test tells both
the same points, so every refit sees identical data.

Tolerances (stated here, measured in DESIGN §4):
* proposals: integer dimensions exact, real dimensions within ``REAL_TOL``;
* candidate top-5 per acquisition: identical indices (the candidates are the
  same draws; this is the EI/PI/LCB argsort over 10 000 candidates);
* the gp_hedge pick: identical;
* fitted theta (log space): within ``THETA_TOL`` -- sklearn's L-BFGS-B and the
  device-objective L-BFGS-B stop at slightly different points of flat
  directions (length scales at the 100 bound), which moves the posterior far
  less than it moves theta;
* gp_hedge gains (sums of posterior means at the previous proposals): within
  ``GAINS_RTOL`` relative -- they inherit the theta differences (first GPU run:
  up to 9.5e-6 relative, with log-theta within 6.4e-5).
"""
import numpy as np
import pytest

from oracle.skopt_optimizer import SkoptOracle

pytestmark = pytest.mark.gpu

REAL_TOL = 1e-6
THETA_TOL = 1e-3
GAINS_RTOL = 1e-4
# n ~ 200 (the configs[3] search's refit sizes): the LML surface is flat enough that
# sklearn's fit and the device fit stop up to 4e-4 apart in log theta (both inside
# the solver's ftol; measured 3.9e-4 with the native driver, 3.6e-4 with scipy's own
# setulb -- so not the driver), and the acquisition polish (maxiter=20) moves the
# real dimension of a proposal with theta: measured 4.8e-4 with either driver, while
# integer dimensions, every top-5 and every gp_hedge pick stay identical
REAL_TOL_LARGE_N = 1e-3


def f_mnist(x):
    nb, pool, ks, dense, drop = x
    return float(((nb - 30) / 40) ** 2 + ((pool - 4) / 8) ** 2 + ((ks - 5) / 8) ** 2 + ((dense - 120) / 150) ** 2
                 + (drop - 0.3) ** 2 + 0.05 * np.sin(nb * dense / 300.0))


def _same_point(a, b, where, real_tol=REAL_TOL):
    assert len(a) == len(b), where
    for j, (u, v) in enumerate(zip(a, b)):
        if isinstance(v, (int, np.integer)):
            assert int(u) == int(v), f"{where}: dim {j}: {a} vs oracle {b}"
        else:
            assert abs(float(u) - float(v)) <= real_tol, f"{where}: dim {j}: {a} vs oracle {b}"


def _compare_traces(td, to, where):
    assert len(td) == len(to), f"{where}: {len(td)} refits vs oracle {len(to)}"
    worst = {"theta": 0.0, "gains": 0.0}
    for r, (a, b) in enumerate(zip(td, to)):
        th_d = np.log(np.concatenate([[a["theta"][0]], a["theta"][1], [a["theta"][2]]]))
        th_o = np.log(np.concatenate([[b["theta"][0]], b["theta"][1], [b["theta"][2]]]))
        worst["theta"] = max(worst["theta"], float(np.max(np.abs(th_d - th_o))))
        assert np.max(np.abs(th_d - th_o)) <= THETA_TOL, f"{where} refit {r}: theta {th_d} vs oracle {th_o}"
        for acq in b["top"]:
            assert list(a["top"][acq]) == list(b["top"][acq]), f"{where} refit {r} {acq}: top-5 differs"
        assert a["pick"] == b["pick"], f"{where} refit {r}: gp_hedge pick {a['pick']} vs oracle {b['pick']}"
        gd = float(np.max(np.abs(a["gains"] - b["gains"]) / np.maximum(1.0, np.abs(b["gains"])))) if len(b["gains"]) \
            else 0.0
        worst["gains"] = max(worst["gains"], gd)
        assert gd <= GAINS_RTOL, f"{where} refit {r}: gains {a['gains']} vs oracle {b['gains']}"
    return worst


def test_ask_tell_sequence_and_cl_min_batch_match_skopt_oracle():
    from mpi_opt_amd.models import mnist_space
    from mpi_opt_amd.optimizer import Optimizer

    opt = Optimizer(mnist_space(), random_state=13579, device="cuda:0")
    opt.trace = []
    ora = SkoptOracle(mnist_space(), random_state=13579)
    for i in range(20):
        xd, xo = opt.ask(), ora.ask()
        _same_point(xd, xo, f"ask {i}")
        y = f_mnist(xo)
        opt.tell(xo, y)
        ora.tell(xo, y)
    worst = _compare_traces(opt.trace, ora.trace, "tell sequence")
    # the reference's batch: Coordinator.ask -> optimizer.ask(num_iterations) (cl_min lies)
    bd, bo = opt.ask(5), ora.ask(5)
    for k, (a, b) in enumerate(zip(bd, bo)):
        _same_point(a, b, f"cl_min batch point {k}")
    w2 = _compare_traces(opt.batch_trace, ora.batch_trace, "cl_min batch")
    print(f"G2 parity: {len(opt.trace) + len(opt.batch_trace)} refits; max |log theta - oracle| = "
          f"{max(worst['theta'], w2['theta']):.2e}, max gains rel diff = {max(worst['gains'], w2['gains']):.2e}")
    # the cache: a second ask(5) returns the same batch, a tell clears it
    assert opt.ask(5) is bd


def _space_points(n, seed):
    """n points of option3's mnist space from their own RandomState (not the
    optimizers' stream): integer dims as ints, the dropout as a float."""
    rng = np.random.RandomState(seed)
    return [[int(rng.randint(10, 51)), int(rng.randint(2, 11)), int(rng.randint(2, 11)), int(rng.randint(50, 201)),
             float(rng.uniform(0.0, 1.0))] for _ in range(n)]


@pytest.mark.parametrize("driver", ["native", "scipy"])
@pytest.mark.parametrize("n_told", [200])
def test_ask_tell_at_search_sizes_match_skopt_oracle(n_told, driver, monkeypatch):
    """G2 where the configs[3] search runs (refits at n = 64 ... 447, mean 223, DESIGN
    §3.1c): both optimizers are told the same ``n_told`` points at once (one refit at
    n = n_told), then three ask/tell rounds (n_told + 1 ... + 3), then the reference's
    ``ask(5)`` cl_min batch (copy() refit + 4 lie refits past it).  With either
    L-BFGS-B driver (``optimizer.DRIVER``: the native csrc/lbfgsb.cpp default, or
    scipy's own setulb), every refit's fitted theta, candidate top-5 per acquisition,
    gp_hedge pick and gains must match the oracle (sklearn's own fit + scipy polish)
    with the tolerances above; proposals: integer dimensions exact, the real one
    within REAL_TOL_LARGE_N."""
    from mpi_opt_amd import optimizer as OPT
    from mpi_opt_amd.models import mnist_space
    from mpi_opt_amd.optimizer import Optimizer

    monkeypatch.setattr(OPT, "DRIVER", driver)
    opt = Optimizer(mnist_space(), random_state=13579, device="cuda:0")
    opt.trace = []
    ora = SkoptOracle(mnist_space(), random_state=13579)
    X = _space_points(n_told, 7)
    Y = [f_mnist(x) for x in X]
    opt.tell(X, Y)
    ora.tell(X, Y)
    asked = []
    for i in range(3):
        xd, xo = opt.ask(), ora.ask()
        asked.append((xd, xo))
        y = f_mnist(xo)
        opt.tell(xo, y)
        ora.tell(xo, y)
    bd, bo = opt.ask(5), ora.ask(5)
    # the refits first (theta, top-5, picks, gains): a proposal inherits their differences
    worst = _compare_traces(opt.trace, ora.trace, f"{driver}: tells at n={n_told}..{n_told + 3}")
    w2 = _compare_traces(opt.batch_trace, ora.batch_trace, f"{driver}: cl_min batch")
    real = max(abs(float(a[4]) - float(b[4])) for a, b in asked + list(zip(bd, bo)))
    print(f"G2 parity at n={n_told} ({driver}): {len(opt.trace) + len(opt.batch_trace)} refits; max |log theta - "
          f"oracle| = {max(worst['theta'], w2['theta']):.2e}, max gains rel diff = "
          f"{max(worst['gains'], w2['gains']):.2e}, max real-dim proposal diff = {real:.2e}")
    for i, (xd, xo) in enumerate(asked):
        _same_point(xd, xo, f"{driver} n={n_told + i}: ask {i}", REAL_TOL_LARGE_N)
    for k, (a, b) in enumerate(zip(bd, bo)):
        _same_point(a, b, f"{driver}: cl_min batch point {k} (n={n_told + 3 + k})", REAL_TOL_LARGE_N)
