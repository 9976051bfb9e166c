"""GP hyper-parameter refit, CPU side: the oracle's LML restatement is pinned to
sklearn's own outputs (golden ``gp_lml.npz``), and the lockstep restart driver
(``mpi_opt_amd.gp_fit.lockstep_lbfgsb``) reproduces sklearn's fit exactly when
driven by that objective."""
import os

import numpy as np
import pytest

from oracle import gp_ei as O
from tests.conftest import ROOT

G = np.load(os.path.join(ROOT, "tests", "golden", "gp_lml.npz"))
CASES = ["n200_d10", "n12_d5", "n57_d3", "n230_d4", "n130_d6"]


@pytest.mark.parametrize("name", CASES)
def test_oracle_lml_grad_pinned_to_sklearn(name):
    X, y = G[name + "_X"], G[name + "_y"]
    for t, lml, grad in zip(G[name + "_theta"], G[name + "_lml"], G[name + "_grad"]):
        v, g = O.lml_and_grad(X, y, t)
        assert abs(v - lml) <= 1e-9 * abs(lml)
        assert np.max(np.abs(g - grad)) <= 1e-8 * max(1.0, np.max(np.abs(grad)))


def _oracle_batch(X, y):
    def ev(T):
        out = [O.lml_and_grad(X, y, t) for t in T]
        return np.array([o[0] for o in out]), np.stack([o[1] for o in out]), np.zeros(len(T), np.int32)
    return ev


@pytest.mark.parametrize("name", ["n12_d5", "n57_d3"])
def test_lockstep_restarts_reproduce_sklearn_fit(name):
    from mpi_opt_amd.gp_fit import lockstep_lbfgsb

    X, y, d = G[name + "_X"], G[name + "_y"], G[name + "_X"].shape[1]
    (amp, ls, noise), det = lockstep_lbfgsb(_oracle_batch(X, y), d, random_state=int(G[name + "_seed"]),
                                            return_details=True)
    theta = np.log(np.r_[amp, ls, noise])
    assert np.allclose(theta, G[name + "_fit_theta"], rtol=0, atol=1e-6)
    assert abs(det["lml"] - float(G[name + "_fit_lml"])) <= 1e-8 * abs(float(G[name + "_fit_lml"]))
    # every evaluation of all three restarts went through a shared batch
    assert det["launches"] < sum(1 for _ in det["optima"]) * 200


def test_lockstep_propagates_objective_errors():
    from mpi_opt_amd.gp_fit import lockstep_lbfgsb

    def bad(T):
        raise RuntimeError("device failure")

    with pytest.raises(RuntimeError, match="device failure"):
        lockstep_lbfgsb(bad, 3, random_state=0)


def test_batched_reverse_communication_lbfgsb_is_scipys_path():
    """lbfgsb_batched (one thread, scipy's setulb in reverse communication, the
    runs' evaluations batched per round) reproduces scipy.optimize.minimize
    (L-BFGS-B, the GP refit) and fmin_l_bfgs_b(maxiter=20) (the acquisition
    polish) bit for bit, run by run."""
    import scipy.optimize
    from scipy.optimize import fmin_l_bfgs_b

    from mpi_opt_amd import gp_fit as GF

    assert GF._setulb() is not None
    X, y = O.synthetic_problem(40, 5, seed=3)
    d = 5
    bounds = GF.theta_bounds(d)
    rng = np.random.RandomState(0)
    starts = [np.zeros(d + 2)] + [rng.uniform(bounds[:, 0], bounds[:, 1]) for _ in range(2)]

    def ev(T, ids):
        out = [O.lml_and_grad(X, y, t) for t in T]
        return np.array([-v for v, _ in out]), np.array([-g for _, g in out])

    got, rounds = GF.lbfgsb_batched(ev, starts, bounds)
    nfev = []
    for s0, (x, f) in zip(starts, got):
        r = scipy.optimize.minimize(lambda t: tuple(-np.asarray(v) for v in O.lml_and_grad(X, y, t)), s0,
                                    method="L-BFGS-B", jac=True, bounds=bounds)
        assert np.array_equal(r.x, x) and r.fun == f
        nfev.append(r.nfev)
    assert rounds == max(nfev)

    st = O.gp_from_theta(X, y, 1.3, np.full(d, 0.5), 1e-3)
    ps = [rng.uniform(size=d) for _ in range(5)]

    def ev2(P, ids):
        out = [O.acquisition_and_grad(st, p, float(y.min()), "EI") for p in P]
        return np.array([v for v, _ in out]), np.array([g for _, g in out])

    got, _ = GF.lbfgsb_batched(ev2, ps, [(0.0, 1.0)] * d, ftol=GF.FMIN_FTOL, maxiter=20)
    for p0, (x, f) in zip(ps, got):
        xr, fr, _ = fmin_l_bfgs_b(lambda v: O.acquisition_and_grad(st, v, float(y.min()), "EI"), p0,
                                  bounds=[(0.0, 1.0)] * d, approx_grad=False, maxiter=20)
        assert np.array_equal(xr, x) and fr == f
