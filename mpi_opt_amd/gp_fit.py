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
        self._cap = 0

    def _ensure(self, batch):
        if batch <= self._cap:
            return
        L = _lib.lib()
        self.ws_bytes = int(L.mpo_gp_lml_ws_bytes(self.n, self.d, batch))
        if self.ws_bytes == 0:
            raise _lib.MpoError(f"mpo_gp_lml_grad: n={self.n} d={self.d} unsupported")
        self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)
        self.theta_d = torch.empty((batch, self.d + 2), dtype=torch.float64, device=self.device)
        # lml | grad | info in ONE device buffer: one device-to-host copy (one sync)
        # per L-BFGS iteration instead of three
        k = self.d + 2
        self.out_d = torch.empty(batch * (k + 2), dtype=torch.float64, device=self.device)
        self.lml_d = self.out_d[:batch]
        self.grad_d = self.out_d[batch:batch * (k + 1)].view(batch, k)
        self.info_d = self.out_d[batch * (k + 1):].view(torch.int32)[:batch]
        self.theta_h = torch.empty((batch, k), dtype=torch.float64).pin_memory()
        self.out_h = torch.empty(batch * (k + 2), dtype=torch.float64).pin_memory()
        self._cap = batch

    def evaluate(self, thetas):
        """thetas [B, d+2] (log space) -> (lml [B], grad [B, d+2], info [B]) as numpy."""
        thetas = np.ascontiguousarray(np.atleast_2d(np.asarray(thetas, dtype=np.float64)))
        B = thetas.shape[0]
        if thetas.shape[1] != self.d + 2:
            raise ValueError(f"theta has {thetas.shape[1]} entries, expected d+2={self.d + 2}")
        # runs on the lockstep worker threads, whose current HIP device is the
        # thread-local default: pin this objective's device for the launch
        with torch.cuda.device(self.device):
            self._ensure(B)
            k, cap = self.d + 2, self._cap
            self.theta_h[:B].numpy()[:] = thetas
            self.theta_d[:B].copy_(self.theta_h[:B], non_blocking=True)
            _lib.check(_lib.lib().mpo_gp_lml_grad(
                _lib.ptr(self.X), _lib.ptr(self.y), self.n, self.d, _lib.ptr(self.theta_d), B,
                _lib.ptr(self.lml_d), _lib.ptr(self.grad_d), _lib.ptr(self.info_d),
                _lib.ptr(self.ws), self.ws_bytes, _lib.stream_handle(self.device)), "mpo_gp_lml_grad")
            self.out_h.copy_(self.out_d)          # synchronising copy of all outputs
            h = self.out_h.numpy()
            return (h[:B].copy(), h[cap:cap + B * k].reshape(B, k).copy(),
                    h[cap * (k + 1):].view(np.int32)[:B].copy())


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


def fit_lml(X, y, random_state=None, n_restarts_optimizer=2, device=None, return_details=False):
    """skopt's GP refit with the objective on the device.

    Returns (amp, length_scale, noise) -- the fitted ConstantKernel, Matern and
    WhiteKernel parameters, exactly what sklearn's ``kernel_`` would hold -- and,
    with ``return_details``, a dict with the per-start optima and launch count.
    """
    X = np.asarray(X, dtype=np.float64)
    yn, _, _ = normalize_targets(y)
    lml = DeviceLML(X, yn, device=device)
    return lockstep_lbfgsb(lml.evaluate, X.shape[1], random_state, n_restarts_optimizer, return_details)


def lockstep_lbfgsb(evaluate, d, random_state=None, n_restarts_optimizer=2, return_details=False):
    """sklearn's restart loop (_gpr.py:296-337) over a batched objective
    ``evaluate(thetas[B, d+2]) -> (lml[B], grad[B, d+2], info[B])``: the start
    theta and ``n_restarts_optimizer`` uniform draws, L-BFGS-B each (one thread
    per start, evaluations batched in lockstep), best = lowest -lml (first on ties)."""
    bounds = theta_bounds(d)
    rng = check_random_state(random_state)   # GaussianProcessRegressor._rng
    starts = [np.log(np.ones(d + 2))]        # kernel start: amp 1, ls 1, noise 1
    for _ in range(n_restarts_optimizer):
        starts.append(rng.uniform(bounds[:, 0], bounds[:, 1]))

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
    best = int(np.argmin([o[1] for o in optima]))
    theta = np.exp(optima[best][0])
    out = (float(theta[0]), theta[1:d + 1].copy(), float(theta[d + 1]))
    if return_details:
        return out, {"optima": optima, "starts": starts, "launches": step.launches,
                     "lml": -optima[best][1]}
    return out
