"""GP hyper-parameter fit with the log-marginal likelihood evaluated on the GPU.

skopt's ``Optimizer.tell`` refits its surrogate -- sklearn
``GaussianProcessRegressor(kernel=C(1,(0.01,1000)) * Matern(ones(D),(0.01,100),
nu=2.5) + WhiteKernel(), normalize_y=True, n_restarts_optimizer=2)`` -- on every
told point (reached from ``Coordinator.fit``, /root/reference/coordinator.py:63-79).
sklearn's fit (gaussian_process/_gpr.py:296-337) runs L-BFGS-B on
``-log_marginal_likelihood(theta, eval_gradient=True)`` (:537-655) from the
kernel's start theta and from ``n_restarts_optimizer`` draws
``rng.uniform(bounds[:,0], bounds[:,1])``, and keeps the optimum with the lowest
objective (first on ties).

This module keeps that control flow and its arguments, and moves the objective
to ``libmpo.so`` (``mpo_gp_lml_grad``): the restarts run in lockstep (one host
thread each, through :class:`_Lockstep`), so every L-BFGS iteration of all
restarts is ONE launch with one workgroup per theta.  Each theta's result
depends only on that theta (fixed summation order), so batching never changes
an optimisation path.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import scipy.optimize
import torch

from . import _lib
from .space import check_random_state

AMP_BOUNDS = (0.01, 1000.0)    # skopt cook_estimator ConstantKernel(1.0, (0.01, 1000.0))
LS_BOUNDS = (0.01, 100.0)      # Matern(length_scale_bounds=[(0.01, 100)] * D)
NOISE_BOUNDS = (1e-5, 1e5)     # WhiteKernel() defaults (skopt noise="gaussian")


def theta_bounds(d):
    """sklearn ``kernel.bounds`` of skopt's kernel: log of (amp, ls_0..ls_{d-1}, noise)."""
    return np.log(np.array([AMP_BOUNDS] + [LS_BOUNDS] * d + [NOISE_BOUNDS], dtype=np.float64))


def normalize_targets(y):
    """sklearn ``normalize_y``: (y - mean) / std with _handle_zeros_in_scale."""
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    mean = float(np.mean(y))
    std = float(np.std(y))
    if std == 0.0:
        std = 1.0
    return (y - mean) / std, mean, std


class DeviceLML:
    """The LML objective of one training set, resident on one GPU."""

    def __init__(self, X, y_norm, device=None):
        self.device = torch.device(device if device is not None else "cuda")
        X = np.ascontiguousarray(np.asarray(X, dtype=np.float64))
        self.n, self.d = X.shape
        self.X = torch.from_numpy(X).to(self.device)
        self.y = torch.from_numpy(np.ascontiguousarray(y_norm, dtype=np.float64)).to(self.device)
        self._stream = _lib.stream_handle(self.device)
        self._cap = 0

    def _ensure(self, batch):
        if batch <= self._cap:
            return
        L = _lib.lib()
        self.ws_bytes = int(L.mpo_gp_lml_ws_bytes(self.n, self.d, batch))
        if self.ws_bytes == 0:
            raise _lib.MpoError(f"mpo_gp_lml_grad: n={self.n} d={self.d} unsupported")
        self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)
        self.io_bytes = int(L.mpo_gp_lml_io_bytes(self.d, batch))
        self.io = torch.empty(self.io_bytes, dtype=torch.uint8, device=self.device)
        k = self.d + 2
        # device views of the io buffer at full capacity (direct mpo_gp_lml_grad timing in bench / probes)
        io = self.io.view(torch.float64)
        self.theta_d = io[:batch * k].view(batch, k)
        self.lml_d = io[batch * k:batch * (k + 1)]
        self.grad_d = io[batch * (k + 1):batch * (2 * k + 1)].view(batch, k)
        self.info_d = io[batch * (2 * k + 1):].view(torch.int32)[:batch]
        # host side of one round: theta in, lml | grad | info out (pinned)
        self.theta_h = torch.empty((batch, k), dtype=torch.float64).pin_memory()
        self.out_h = torch.empty(batch * (k + 1) + (batch + 1) // 2, dtype=torch.float64).pin_memory()
        self._cap = batch
        # one round's call, its pointers resolved once (a round is ~100-400 us of
        # device time; ctypes argument packing and tensor data_ptr lookups were ~10 us of it)
        self._th_np, self._out_np = self.theta_h.numpy(), self.out_h.numpy()
        fn = L.mpo_gp_lml_grad_host
        args = (_lib.ptr(self.X), _lib.ptr(self.y), self.n, self.d, self.theta_h.data_ptr())
        tail = (self.out_h.data_ptr(), _lib.ptr(self.io), self.io_bytes, _lib.ptr(self.ws), self.ws_bytes, self._stream)
        self._call = lambda B: fn(*args, B, *tail)

    def negated_round(self, thetas, ids=None):
        """(-lml [B], -grad [B, d+2]) for the L-BFGS-B driver: ``thetas`` is its
        C-contiguous float64 [B, d+2] buffer; fresh arrays out."""
        B = len(thetas)
        if B > self._cap:
            self._ensure(B)
        self._th_np[:B] = thetas
        rc = self._call(B)
        if rc != 0:
            _lib.check(rc, "mpo_gp_lml_grad_host")
        h = self._out_np
        return -h[:B], -(h[B:B + B * (self.d + 2)].reshape(B, self.d + 2))

    def fit(self, starts, bounds, ftol=None, gtol=1e-5, maxiter=15000, maxfun=15000, batcher=True):
        """L-BFGS-B from every start on -LML, all in ``mpo_gp_fit_lml_host`` (the
        host L-BFGS-B of csrc/lbfgsb.cpp; one device round per iteration of all
        live runs; ctypes releases the GIL for the whole fit).  The rounds go
        through the device's batcher (``_lib.lml_batcher``): concurrent fits on
        this GPU (the cl_min chains) share launches, with unchanged results.
        ``batcher=False`` runs every round on this fit's own stream instead (the
        plain per-round path; the tests' baseline).
        Returns ([(theta, -lml)] per start, rounds)."""
        starts = np.ascontiguousarray(np.asarray(starts, dtype=np.float64))
        B, k = starts.shape
        if k != self.d + 2:
            raise ValueError(f"theta has {k} entries, expected d+2={self.d + 2}")
        self._ensure(B)
        b = np.ascontiguousarray(np.asarray(bounds, dtype=np.float64).reshape(k, 2))
        opts = _lib.MpoLbfgsbOptions(MINIMIZE_FTOL if ftol is None else ftol, gtol, maxiter, maxfun, 10, 20)
        x = np.empty((B, k))
        f = np.empty(B)
        stats = np.empty((B, 4), np.int32)
        rounds = ctypes.c_int32(0)
        rc = _lib.lib().mpo_gp_fit_lml_host(
            _lib.ptr(self.X), _lib.ptr(self.y), self.n, self.d, starts.ctypes.data, B, b.ctypes.data,
            ctypes.byref(opts), self.theta_h.data_ptr(), self.out_h.data_ptr(), _lib.ptr(self.io), self.io_bytes,
            _lib.ptr(self.ws), self.ws_bytes, x.ctypes.data, f.ctypes.data, stats.ctypes.data, ctypes.byref(rounds),
            _lib.lml_batcher(self.X.device.index) if batcher else None, self._stream)
        _lib.check(rc, "mpo_gp_fit_lml_host")
        self.last_stats = stats
        return [(x[r], float(f[r])) for r in range(B)], rounds.value

    def evaluate(self, thetas):
        """thetas [B, d+2] (log space) -> (lml [B], grad [B, d+2], info [B]) as numpy:
        one ``mpo_gp_lml_grad_host`` call (copy in, objective, copy out, sync)."""
        thetas = np.asarray(thetas, dtype=np.float64)
        if thetas.ndim == 1:
            thetas = thetas[None, :]
        B = thetas.shape[0]
        if thetas.shape[1] != self.d + 2:
            raise ValueError(f"theta has {thetas.shape[1]} entries, expected d+2={self.d + 2}")
        self._ensure(B)
        k = self.d + 2
        self._th_np[:B] = thetas
        rc = self._call(B)
        if rc != 0:
            _lib.check(rc, "mpo_gp_lml_grad_host")
        h = self._out_np
        return (h[:B].copy(), h[B:B + B * k].reshape(B, k).copy(), h[B + B * k:].view(np.int32)[:B].copy())


# scipy's L-BFGS-B defaults as ``minimize(method="L-BFGS-B")`` and ``fmin_l_bfgs_b`` pass them
MINIMIZE_FTOL = 2.2204460492503131e-09
FMIN_FTOL = 1e7 * np.finfo(float).eps      # fmin_l_bfgs_b: factr=1e7 -> ftol = factr * eps


def _setulb():
    try:
        from scipy.optimize import _lbfgsb
        return _lbfgsb.setulb if "ln_task" in (_lbfgsb.setulb.__doc__ or "") else None
    except ImportError:      # pragma: no cover -- another scipy: the threaded driver below is used
        return None


class _LbfgsbRun:
    """One L-BFGS-B minimisation in reverse communication, step for step what
    scipy 1.15's ``_minimize_lbfgsb`` does around ``_lbfgsb.setulb`` (with its
    ``ScalarFunction`` cache: the objective is evaluated at the clipped x0 first,
    and an FG request at an unchanged x reuses that value)."""

    def __init__(self, x0, bounds, ftol, gtol, maxiter, maxfun, maxcor=10, maxls=20):
        lo, hi = np.asarray(bounds, dtype=np.float64).T
        self.x = np.clip(np.asarray(x0, dtype=np.float64).ravel(), lo, hi).astype(np.float64)
        n = self.x.size
        self.m, self.maxls, self.maxiter, self.maxfun = maxcor, maxls, maxiter, maxfun
        self.factr, self.pgtol = ftol / np.finfo(float).eps, gtol
        self.low, self.up = lo.copy(), hi.copy()
        self.nbd = np.full(n, 2, dtype=np.int32)          # both bounds finite (every bound here is)
        self.f = np.array(0.0, dtype=np.int32)
        self.g = np.zeros((n,), dtype=np.int32)
        self.wa = np.zeros(2 * maxcor * n + 5 * n + 11 * maxcor * maxcor + 8 * maxcor, np.float64)
        self.iwa = np.zeros(3 * n, dtype=np.int32)
        self.task = np.zeros(2, dtype=np.int32)
        self.ln_task = np.zeros(2, dtype=np.int32)
        self.lsave = np.zeros(4, dtype=np.int32)
        self.isave = np.zeros(44, dtype=np.int32)
        self.dsave = np.zeros(29, dtype=np.float64)
        self.nit = 0
        self.nfev = 0
        self.sf_x = None          # ScalarFunction's cached point and values
        self.sf_f = self.sf_g = None
        self.started = False
        self.done = False

    def request(self):
        """The first evaluation (ScalarFunction at x0): x to evaluate."""
        return self.x.copy()

    def deliver(self, x, f, g):
        """f, g at x: into the ScalarFunction cache and, once setulb has asked for
        them (every delivery after the first), into the run."""
        self.sf_x, self.sf_f, self.sf_g = x, f, g
        self.nfev += 1
        if self.started:
            self.f, self.g = f, g
        self.started = True

    def advance(self, setulb):
        """Run setulb until it needs f, g at a new point (returns that point) or
        stops (returns None)."""
        task = self.task
        while True:
            if self.g.dtype != np.float64:     # scipy's g.astype(np.float64); deliver() hands float64 already
                self.g = self.g.astype(np.float64)
            setulb(self.m, self.x, self.low, self.up, self.nbd, self.f, self.g, self.factr, self.pgtol, self.wa,
                   self.iwa, task, self.lsave, self.isave, self.dsave, self.maxls, self.ln_task)
            t0 = task[0]
            if t0 == 3:
                # ScalarFunction's cache: the same x (np.array_equal of same-shape float
                # arrays: elementwise ==, so -0.0 == 0.0 and NaN != NaN -- as Python float
                # equality on fresh float objects, ~10x cheaper than the ufunc reduction)
                if self.sf_x is not None and self.x.tolist() == self.sf_x.tolist():
                    self.f, self.g = self.sf_f, self.sf_g
                    continue
                return self.x.copy()
            if t0 == 1:
                self.nit += 1
                if self.nit >= self.maxiter:
                    task[0], task[1] = 5, 504
                elif self.nfev > self.maxfun:
                    task[0], task[1] = 5, 502
                continue
            self.done = True
            return None


def lbfgsb_batched(evaluate, starts, bounds, ftol=MINIMIZE_FTOL, gtol=1e-5, maxiter=15000, maxfun=15000):
    """Independent L-BFGS-B runs from ``starts`` whose objective evaluations are
    batched: every round calls ``evaluate(X[B, n], ids) -> (f[B], g[B, n])`` once
    with the point each live run needs.  One thread drives every run through
    scipy's reverse-communication ``setulb`` exactly as ``scipy.optimize.minimize
    (method="L-BFGS-B", jac=True)`` (``ftol=MINIMIZE_FTOL``) or ``fmin_l_bfgs_b``
    (``ftol=FMIN_FTOL``) would, so each run's iterates are those of a sequential
    scipy call.  Returns ([(x, f)] per run, number of rounds).

    The loop holds the GIL between the device rounds (concurrent cl_min chains,
    mpi_opt_amd.chains, share it): the _LbfgsbRun protocol (deliver, then
    advance) is inlined and the rows of ``g`` are handed to the runs without a
    copy, so ``evaluate`` must return fresh arrays.  (r05: ~18 us of host time per
    round of 3 runs on the GPU box, scripts/lbfgs_host_bench.py, the same as the
    method-per-run form; the cProfile'd chain makes a third fewer Python calls.)"""
    setulb = _setulb()
    runs = [_LbfgsbRun(x0, bounds, ftol, gtol, maxiter, maxfun) for x0 in starts]
    r0 = runs[0]
    m, low, up, nbd, factr, pgtol, maxls = r0.m, r0.low, r0.up, r0.nbd, r0.factr, r0.pgtol, r0.maxls
    live = list(range(len(runs)))
    want = [r.request() for r in runs]
    buf = np.empty((len(runs), r0.x.size), dtype=np.float64)   # the round's points (no np.stack)
    rounds = 0
    while live:
        nl = len(live)
        X = buf[:nl]
        for k in range(nl):
            X[k] = want[live[k]]
        f, g = evaluate(X, live)
        rounds += 1
        nxt = []
        for k in range(nl):
            i = live[k]
            r = runs[i]
            # deliver: the ScalarFunction cache, then (after the first) the run's f, g
            x = want[i]
            fk, gk = float(f[k]), g[k]
            r.sf_x, r.sf_f, r.sf_g = x, fk, gk
            sfx = x.tolist()
            r.nfev += 1
            if r.started:
                r.f, r.g = fk, gk
            r.started = True
            # advance: setulb until it asks for f, g at a new point or stops
            task, rx = r.task, r.x
            while True:
                rg = r.g
                if rg.dtype != np.float64:      # scipy's g.astype(np.float64) (the START call only)
                    rg = r.g = rg.astype(np.float64)
                setulb(m, rx, low, up, nbd, r.f, rg, factr, pgtol, r.wa, r.iwa, task, r.lsave, r.isave, r.dsave,
                       maxls, r.ln_task)
                t0 = task[0]
                if t0 == 3:
                    if rx.tolist() == sfx:      # ScalarFunction's cache: the same x (elementwise ==)
                        r.f, r.g = r.sf_f, r.sf_g
                        continue
                    want[i] = rx.copy()
                    nxt.append(i)
                    break
                if t0 == 1:
                    r.nit += 1
                    if r.nit >= r.maxiter:
                        task[0], task[1] = 5, 504
                    elif r.nfev > r.maxfun:
                        task[0], task[1] = 5, 502
                    continue
                r.done = True
                break
        live = nxt
    return [(r.x, float(r.f)) for r in runs], rounds


class _Lockstep:
    """Collects one theta from every live optimiser thread, evaluates them in one
    batch, hands each thread its own result."""

    def __init__(self, evaluate, n_workers, pass_ids=False):
        self.evaluate = evaluate
        self.pass_ids = pass_ids
        self.cv = threading.Condition()
        self.active = n_workers
        self.pending = {}
        self.results = {}
        self.launches = 0

    def __call__(self, wid, theta):
        with self.cv:
            self.pending[wid] = np.array(theta, dtype=np.float64)
            self._flush()
            while wid not in self.results:
                self.cv.wait()
            r = self.results.pop(wid)
        if isinstance(r, BaseException):
            raise r
        return r

    def retire(self):
        with self.cv:
            self.active -= 1
            self._flush()

    def _flush(self):  # lock held
        if not self.pending or len(self.pending) < self.active:
            return
        ids = sorted(self.pending)
        thetas = np.stack([self.pending[i] for i in ids])
        self.pending = {}
        try:
            out = self.evaluate(thetas, ids) if self.pass_ids else self.evaluate(thetas)
            val, grad = out[0], out[1]
            self.launches += 1
            for k, i in enumerate(ids):
                self.results[i] = (float(val[k]), grad[k].copy())
        except BaseException as e:  # every waiting thread re-raises
            for i in ids:
                self.results[i] = e
        self.cv.notify_all()


def fit_lml(X, y, random_state=None, n_restarts_optimizer=2, device=None, return_details=False, driver="native"):
    """skopt's GP refit with the objective on the device.

    Returns (amp, length_scale, noise) -- the fitted ConstantKernel, Matern and
    WhiteKernel parameters, exactly what sklearn's ``kernel_`` would hold -- and,
    with ``return_details``, a dict with the per-start optima and launch count.
    ``driver``: "native" runs L-BFGS-B in libmpo.so (``DeviceLML.fit``, no GIL
    held during the fit); "scipy" drives scipy's own setulb from Python
    (``lbfgsb_batched``: scipy's iterates bit for bit, given the objective).
    """
    X = np.asarray(X, dtype=np.float64)
    yn, _, _ = normalize_targets(y)
    lml = DeviceLML(X, yn, device=device)
    return lockstep_lbfgsb(lml.evaluate, X.shape[1], random_state, n_restarts_optimizer, return_details, driver)


def lockstep_lbfgsb(evaluate, d, random_state=None, n_restarts_optimizer=2, return_details=False, driver="native"):
    """sklearn's restart loop (_gpr.py:296-337) over a batched objective
    ``evaluate(thetas[B, d+2]) -> (lml[B], grad[B, d+2], info[B])``: the start
    theta and ``n_restarts_optimizer`` uniform draws, L-BFGS-B each (one thread
    per start, evaluations batched in lockstep), best = lowest -lml (first on ties).
    A ``DeviceLML.evaluate`` objective with ``driver="native"`` runs the whole
    fit in ``mpo_gp_fit_lml_host``."""
    bounds = theta_bounds(d)
    rng = check_random_state(random_state)   # GaussianProcessRegressor._rng
    starts = [np.log(np.ones(d + 2))]        # kernel start: amp 1, ls 1, noise 1
    for _ in range(n_restarts_optimizer):
        starts.append(rng.uniform(bounds[:, 0], bounds[:, 1]))

    fast = getattr(evaluate, "__self__", None)
    if driver == "native" and isinstance(fast, DeviceLML):
        optima, launches = fast.fit(np.array(starts), bounds)
        return _pick(optima, starts, launches, d, return_details)
    if driver not in ("native", "scipy"):
        raise ValueError(f"driver {driver!r}: 'native' or 'scipy'")

    if _setulb() is not None:                # one thread, setulb in reverse communication
        if isinstance(fast, DeviceLML):
            neg = fast.negated_round             # the device round, negated, without the checks
        else:
            def neg(thetas, ids):
                v, g = evaluate(thetas)[:2]
                return -np.asarray(v), -np.asarray(g)
        optima, launches = lbfgsb_batched(neg, starts, bounds)
        return _pick(optima, starts, launches, d, return_details)

    step = _Lockstep(evaluate, len(starts))
    optima = [None] * len(starts)
    errors = []

    def run(wid):
        try:
            def obj(theta):
                v, g = step(wid, theta)
                return -v, -g
            res = scipy.optimize.minimize(obj, starts[wid], method="L-BFGS-B", jac=True, bounds=bounds)
            optima[wid] = (res.x, float(res.fun))
        except BaseException as e:  # noqa: BLE001 -- re-raised on the caller's thread
            errors.append(e)
        finally:
            step.retire()

    threads = [threading.Thread(target=run, args=(w,), daemon=True) for w in range(len(starts))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return _pick(optima, starts, step.launches, d, return_details)


def _pick(optima, starts, launches, d, return_details):
    """sklearn: the optimum with the lowest -LML, first on ties (_gpr.py:331-333)."""
    best = int(np.argmin([o[1] for o in optima]))
    theta = np.exp(optima[best][0])
    out = (float(theta[0]), theta[1:d + 1].copy(), float(theta[d + 1]))
    if return_details:
        return out, {"optima": optima, "starts": starts, "launches": launches, "lml": -optima[best][1]}
    return out
