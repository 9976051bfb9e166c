"""Pin the GP/EI oracle (oracle/gp_ei.py) against sklearn 1.7.2 -- the arithmetic
base scikit-optimize subclasses -- and against the committed golden fixtures."""
import glob
import os

import numpy as np
import pytest

from oracle import gp_ei as O
from tests.conftest import GOLDEN

FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "gp_ei_*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def state(f):
    return O.gp_from_theta(f["X"], f["y"], float(f["amp"]), f["ls"], float(f["noise"]))


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_cholesky_and_alpha_match_sklearn(path):
    f = load(path)
    st = state(f)
    np.testing.assert_allclose(st.L, f["sk_L"], rtol=1e-11, atol=1e-13)
    np.testing.assert_allclose(st.alpha, f["sk_alpha"], rtol=1e-9, atol=1e-9 * np.abs(f["sk_alpha"]).max())


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_posterior_pinned_to_sklearn_predict(path):
    f = load(path)
    st = state(f)
    mu, sd = O.posterior_skopt(st, f["C"])
    np.testing.assert_allclose(mu, f["mu"], rtol=0, atol=1e-12 * st.y_std * (1 + np.abs(mu).max()))
    np.testing.assert_allclose(sd, f["sd"], rtol=1e-12)
    # sklearn's V-solve predict and the 80-bit restatement agree to ~1e-11
    assert np.max(np.abs(f["sk_sd"] - f["sd_exact"]) / f["sd_exact"]) < 1e-10
    scale = st.y_std * (np.abs(O.matern52(f["C"], st.X, st.length_scale, st.amp)) @ np.abs(st.alpha)) + abs(st.y_mean)
    assert np.max(np.abs(f["sk_mu"] - f["mu_exact"]) / scale) < 1e-12
    # skopt's einsum sd sits within its own rounding bound of the exact posterior
    eps = np.finfo(np.float64).eps
    dvar = 4 * np.sqrt(st.n) * eps * f["qbound"]
    bound = 1e-12 * f["sd_exact"] + st.y_std ** 2 * dvar / (2 * f["sd_exact"])
    assert np.all(np.abs(f["sd"] - f["sd_exact"]) <= bound)


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_acquisitions_and_argmins(path):
    f = load(path)
    for acq in ("EI", "PI", "LCB"):
        v = O.acquisition_values(f["mu"], f["sd"], float(f["y_opt"]), acq, float(f["xi"]), float(f["kappa"]))
        np.testing.assert_array_equal(v, f["v_" + acq])
        assert O.argmin_lowest(v) == int(f["argmin_" + acq])
        np.testing.assert_array_equal(O.topk_lowest(v, 5), f["top5_" + acq])
    assert f["ei_top2_relgap"] > 1e-6


def test_ei_matches_closed_form_and_masks_zero_std():
    mu = np.array([0.0, 1.0, -1.0, 0.5])
    sd = np.array([1.0, 0.0, 2.0, 1e-3])
    v = O.gaussian_ei(mu, sd, y_opt=0.2, xi=0.01)
    assert v[1] == 0.0
    from scipy.stats import norm
    z = (0.2 - 0.01 - mu[0]) / sd[0]
    assert abs(v[0] - ((0.19) * norm.cdf(z) + norm.pdf(z))) < 1e-15


def test_argmin_ties_lowest_index():
    v = np.array([3.0, -1.0, 2.0, -1.0, -1.0])
    assert O.argmin_lowest(v) == 1
    assert list(O.topk_lowest(v, 3)) == [1, 3, 4]


@pytest.mark.slow
def test_refit_reproduces_fixture_theta():
    f = load(os.path.join(GOLDEN, "gp_ei_n57_d3.npz"))
    st, _ = O.fit_skopt_gp(f["X"], f["y"], random_state=5)
    assert abs(st.amp - float(f["amp"])) / float(f["amp"]) < 1e-6
    np.testing.assert_allclose(st.length_scale, f["ls"], rtol=1e-6)
