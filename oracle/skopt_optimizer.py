"""CPU oracle for the skopt ``Optimizer`` ask/tell loop.

TEST INFRASTRUCTURE ONLY.  Only ``tests/`` and ``bench.py``'s ``cpu_baseline``
legs may import this module, and only as the checker.  The product path
(``mpi_opt_amd``) never imports it.

What it restates
----------------
The reference builds ``skopt.Optimizer(dimensions=..., random_state=13579)``
(/root/reference/coordinator.py:33), refits it with ``tell(X, Y)`` (:69) and
asks for constant-liar batches with ``ask(num_iterations)`` (:49).
scikit-optimize is un-vendored and unpinned; its published
``Optimizer`` (skopt/optimizer/optimizer.py, 0.8/0.9 line) is restated here on
the pieces this container CAN pin:

* the surrogate fit is sklearn 1.7.2's own ``GaussianProcessRegressor.fit``
  (through :func:`oracle.gp_ei.fit_skopt_gp`: ``C*Matern52 + White``,
  ``normalize_y``, ``n_restarts_optimizer=2``, ``random_state`` = the seed
  ``cook_estimator`` drew once at construction), with skopt's post-fit deltas
  (white noise zeroed, ``K_inv_``);
* the posterior / acquisition values / gradients are :mod:`oracle.gp_ei`
  (pinned to sklearn ``predict`` in ``tests/test_oracle_gp.py``);
* the acquisition polish is scipy's ``fmin_l_bfgs_b(gaussian_acquisition_1D,
  x0, bounds=[0,1]^D, approx_grad=False, maxiter=20)`` from the
  ``np.argsort(values)[:5]`` candidates, as skopt runs it.

The control flow restated on top (parity with skopt itself is UNPINNED: skopt
is absent everywhere here):

* ``__init__``: ``rng = check_random_state(random_state)``; the GP's seed
  ``rng.randint(0, 2**31-1)`` drawn once (``cook_estimator(random_state=...)``);
  ``initial_point_generator="random"`` draws nothing more;
* ``_ask``: random points (``space.rvs(random_state=rng)``) while fewer than
  ``n_initial_points`` were told, then the cached ``_next_x``;
* ``_tell`` with fit: refit; ``gains_ -= est.predict(vstack(next_xs_))`` when a
  previous proposal exists (gp_hedge); ``n_points`` candidates
  ``space.transform(space.rvs(n_points, rng))``; per acquisition in
  [EI, LCB, PI] the polish above, best polished point by ``np.argmin``
  (clipped to [0,1]); gp_hedge picks
  ``next_xs_[argmax(rng.multinomial(1, softmax(eta*gains)))]``;
* ``ask(n, "cl_min")``: ``opt = self.copy(random_state=rng.randint(0,
  2**31-1))`` (the copy re-tells every point, refitting once, and inherits
  ``gains_``), then n times ``x = opt.ask(); opt._tell(x, min(opt.yi))``; the
  batch is cached until the next tell.

Only ``Real``/``Integer`` dimensions with the uniform prior are restated (the
mnist space of option3:126-133 and every BASELINE config use only those).
"""
from __future__ import annotations

import warnings

import numpy as np
from scipy.optimize import fmin_l_bfgs_b

from . import gp_ei as O

INT32_MAX = np.iinfo(np.int32).max


class Dim:
    """skopt ``Real``/``Integer`` after ``normalize_dimensions`` (transform="normalize")."""

    def __init__(self, low, high, integer):
        self.low, self.high, self.integer = low, high, integer

    def rvs(self, n, rng):
        # _uniform_inclusive(0, 1): scipy uniform(loc=0, scale=nextafter(1, 2))
        u = rng.uniform(0.0, np.nextafter(1.0, 2.0), size=n)
        return self.inverse(u)

    def transform(self, x):
        x = np.asarray(x, dtype=float)
        if self.integer:
            return (np.round(x) - self.low) / (self.high - self.low)
        return (x - self.low) / (self.high - self.low)

    def inverse(self, xt):
        x = np.asarray(xt, dtype=float) * (self.high - self.low) + self.low
        if self.integer:
            return np.clip(np.round(x), self.low, self.high).astype(np.int64)
        return np.clip(x, self.low, self.high)


def dims_from(dimensions):
    """(lo, hi) tuples (ints -> Integer) or objects with low/high and an int dtype."""
    out = []
    for d in dimensions:
        if isinstance(d, tuple):
            lo, hi = d
            out.append(Dim(lo, hi, isinstance(lo, (int, np.integer)) and isinstance(hi, (int, np.integer))))
        else:
            out.append(Dim(d.low, d.high, type(d).__name__ == "Integer"))
    return out


class OracleSpace:
    def __init__(self, dims):
        self.dims = dims

    def rvs(self, n, rng):
        cols = [d.rvs(n, rng) for d in self.dims]      # column by column from one stream
        return [[c[i].item() for c in cols] for i in range(n)]

    def transform(self, X):
        X = [list(x) for x in X]
        return np.column_stack([d.transform([x[j] for x in X]) for j, d in enumerate(self.dims)])

    def inverse(self, xt):
        return [d.inverse(xt[j]).item() for j, d in enumerate(self.dims)]


class SkoptOracle:
    """skopt ``Optimizer(dimensions, random_state)`` with the GP defaults."""

    def __init__(self, dimensions, random_state=None, n_initial_points=10, acq_func="gp_hedge", n_points=10000,
                 n_restarts_optimizer=5, xi=0.01, kappa=1.96, eta=1.0, _gp_seed=None):
        self.dimensions = dimensions
        self.space = OracleSpace(dims_from(dimensions))
        self.rng = np.random.RandomState(random_state) if not isinstance(random_state, np.random.RandomState) \
            else random_state
        self.n_initial_points_ = n_initial_points
        self._n_initial_points = n_initial_points
        self.gp_seed = self.rng.randint(0, INT32_MAX) if _gp_seed is None else _gp_seed
        self.acq_func = acq_func
        self.cand_acq_funcs_ = ["EI", "LCB", "PI"] if acq_func == "gp_hedge" else [acq_func]
        if acq_func == "gp_hedge":
            self.gains_ = np.zeros(3)
        self.n_points, self.n_restarts_optimizer = n_points, n_restarts_optimizer
        self.xi, self.kappa, self.eta = xi, kappa, eta
        self.Xi, self.yi, self.models = [], [], []
        self.cache_ = {}
        self.trace = []          # per refit: fitted theta, candidate top-k, polished points, pick

    def copy(self, random_state):
        o = SkoptOracle(self.dimensions, random_state=random_state, n_initial_points=self.n_initial_points_,
                        acq_func=self.acq_func, n_points=self.n_points, n_restarts_optimizer=self.n_restarts_optimizer,
                        xi=self.xi, kappa=self.kappa, eta=self.eta, _gp_seed=self.gp_seed)
        if hasattr(self, "gains_"):
            o.gains_ = np.copy(self.gains_)
        o.trace = []
        if self.Xi:
            o._tell(self.Xi, self.yi)
        return o

    def ask(self, n_points=None):
        if n_points is None:
            return self._ask()
        if n_points in self.cache_:
            return self.cache_[n_points]
        opt = self.copy(random_state=self.rng.randint(0, INT32_MAX))
        X = []
        for _ in range(n_points):
            x = opt.ask()
            X.append(x)
            opt._tell(x, np.min(opt.yi) if opt.yi else 0.0)      # cl_min lie
        self.cache_ = {n_points: X}
        self.batch_trace = opt.trace
        return X

    def _ask(self):
        if self._n_initial_points > 0:
            return self.space.rvs(1, self.rng)[0]
        return self._next_x

    def tell(self, x, y):
        return self._tell(x, y)

    def _tell(self, x, y):
        if np.ndim(y) == 1:
            self.Xi.extend([list(v) for v in x])
            self.yi.extend([float(v) for v in y])
            self._n_initial_points -= len(y)
        else:
            self.Xi.append(list(x))
            self.yi.append(float(y))
            self._n_initial_points -= 1
        self.cache_ = {}
        if self._n_initial_points <= 0:
            self._fit_and_propose()

    def _fit_and_propose(self):
        Xt = self.space.transform(self.Xi)
        y = np.asarray(self.yi, dtype=float)
        with warnings.catch_warnings():          # skopt silences sklearn's ConvergenceWarnings
            warnings.simplefilter("ignore")
            st, _ = O.fit_skopt_gp(Xt, y, random_state=self.gp_seed, n_restarts_optimizer=2)
        if hasattr(self, "next_xs_") and self.acq_func == "gp_hedge":
            self.gains_ -= O.posterior_skopt(st, np.vstack(self.next_xs_))[0]
        self.models.append(st)
        C = self.space.transform(self.space.rvs(self.n_points, self.rng))
        y_opt = float(np.min(self.yi))
        d = C.shape[1]
        bounds = [(0.0, 1.0)] * d
        rec = {"theta": (st.amp, st.length_scale.copy(), st.noise), "top": {}, "polished": {}}
        mu, sd = O.posterior_skopt(st, C)
        self.next_xs_ = []
        for acq in self.cand_acq_funcs_:
            values = O.acquisition_values(mu, sd, y_opt, acq, self.xi, self.kappa)
            x0 = C[np.argsort(values)[:self.n_restarts_optimizer]]
            res = [fmin_l_bfgs_b(lambda v, a=acq: O.acquisition_and_grad(st, v, y_opt, a, self.xi, self.kappa),
                                 x, bounds=bounds, approx_grad=False, maxiter=20) for x in x0]
            xs = np.array([r[0] for r in res])
            fs = np.array([r[1] for r in res])
            rec["top"][acq] = np.argsort(values)[:self.n_restarts_optimizer]
            rec["polished"][acq] = (xs, fs)
            self.next_xs_.append(np.clip(xs[np.argmin(fs)], 0.0, 1.0))
        if self.acq_func == "gp_hedge":
            logits = np.array(self.gains_) - np.max(self.gains_)
            p = np.exp(self.eta * logits)
            p /= p.sum()
            pick = int(np.argmax(self.rng.multinomial(1, p)))
            rec["probs"] = p
        else:
            pick = 0
        rec["pick"] = pick
        rec["gains"] = np.copy(getattr(self, "gains_", np.zeros(0)))
        self.trace.append(rec)
        self._next_x = self.space.inverse(self.next_xs_[pick])
