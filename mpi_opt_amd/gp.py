"""Device-resident GP surrogate: posterior + acquisition scoring on MI355X.

Replaces, for the skopt "gp" base estimator (``cook_estimator("GP")``):

* the tail of ``GaussianProcessRegressor.fit`` -- K, Cholesky ``L_``,
  ``alpha_`` (sklearn/gaussian_process/_gpr.py:345-365) and skopt's post-fit
  white-noise zeroing / ``K_inv_``;
* ``predict(X, return_std=True)`` and ``_gaussian_acquisition`` (EI/PI/LCB)
  over the candidate sample, plus the ``np.argmin`` / ``np.argsort[:k]`` that
  skopt runs on the result.

Reached from ``Coordinator.fit`` / ``Coordinator.ask``
(/root/reference/coordinator.py:63-79, 46-50).  All arithmetic runs in
``libmpo.so`` (fp64); torch is used only to hold device buffers.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr

SKOPT_JITTER = 1e-10


def _dev(device):
    return torch.device(device if device is not None else "cuda")


class DeviceGP:
    """A fitted GP posterior resident on one GPU.

    Parameters mirror the fitted skopt GP: ``X`` observations in the transformed
    space (N, D), raw objective values ``y`` (N,), and kernel hyper-parameters
    ``amp`` (ConstantKernel), ``length_scale`` (Matern, D) and ``noise``
    (WhiteKernel; used in the factorisation, zeroed for prediction as skopt does).
    """

    def __init__(self, X, y, amp, length_scale, noise, device=None):
        self.device = _dev(device)
        X = np.ascontiguousarray(np.asarray(X, dtype=np.float64))
        y = np.asarray(y, dtype=np.float64).reshape(-1)
        if X.ndim != 2 or X.shape[0] != y.shape[0] or X.shape[0] == 0:
            raise ValueError(f"bad GP data shapes X={X.shape} y={y.shape}")
        n, d = X.shape
        ls = np.broadcast_to(np.asarray(length_scale, dtype=np.float64), (d,)).copy()
        # normalize_y=True (sklearn _gpr.py:273-277)
        y_mean = float(np.mean(y))
        y_std = float(np.std(y))
        if y_std == 0.0:
            y_std = 1.0
        y_norm = (y - y_mean) / y_std
        self.n, self.d = n, d
        self.amp, self.noise = float(amp), float(noise)
        self.length_scale = ls
        self.y_mean, self.y_std = y_mean, y_std
        self.y = y
        L = lib()
        self._X = torch.from_numpy(X).to(self.device)
        self._y = torch.from_numpy(y_norm).to(self.device)
        self._ls = torch.from_numpy(ls).to(self.device)
        wsb = L.mpo_gp_prepare_ws_bytes(n, d)
        if wsb == 0:
            raise _lib.MpoError(f"unsupported GP shape n={n} d={d}")
        self._ws = torch.empty(wsb, dtype=torch.uint8, device=self.device)
        self.model = _lib.MpoGpModel()
        with torch.cuda.device(self.device):
            s = _lib.stream_handle(self.device)
            check(L.mpo_gp_prepare(ptr(self._X), ptr(self._y), n, d, ptr(self._ls), self.amp, self.noise,
                                   y_mean, y_std, ctypes.byref(self.model), ptr(self._ws), wsb, s),
                  "mpo_gp_prepare")
        self.chol_info = int(_view_int32(self.model.info, self._ws, self.device).item())
        if self.chol_info != 0:
            raise np.linalg.LinAlgError(
                f"device Cholesky failed at column {self.chol_info - 1} (K not positive definite)")
        self._score_ws = None

    # -- the prepared factor as plain arrays (the sharded scorer's broadcast) ----
    _PTRS = ("xs", "ls", "alpha", "wfrag", "L", "W", "info", "wmeta", "xb")

    def export_factor(self):
        """(meta f64 [3], layout i64 [4 + len(_PTRS)], ws uint8 tensor): everything the
        scoring kernels read, as the prepared workspace plus the offsets of the model's
        pointers into it (-1: NULL).  ``from_factor`` on another GPU rebuilds the
        identical model from a copy of these bytes -- no second factorisation."""
        base = self._ws.data_ptr()
        offs = [(-1 if not getattr(self.model, f) else getattr(self.model, f) - base) for f in self._PTRS]
        layout = np.array([self.model.n, self.model.d, self.model.dp, self.model.np16] + offs, dtype=np.int64)
        meta = np.array([self.model.amp, self.model.y_mean, self.model.y_std], dtype=np.float64)
        return meta, layout, self._ws

    @classmethod
    def from_factor(cls, meta, layout, ws, device=None):
        """A scoring-only DeviceGP over a copy of another rank's prepared workspace
        (``export_factor``): the same model bits, addresses rebased to ``ws``."""
        g = cls.__new__(cls)
        g.device = _dev(device)
        g._ws = ws
        g.model = _lib.MpoGpModel()
        n, d, dp, np16 = (int(v) for v in layout[:4])
        g.model.n, g.model.d, g.model.dp, g.model.np16 = n, d, dp, np16
        g.model.amp, g.model.y_mean, g.model.y_std = (float(v) for v in meta[:3])
        base = ws.data_ptr()
        for f, off in zip(cls._PTRS, layout[4:]):
            setattr(g.model, f, None if int(off) < 0 else base + int(off))
        g.n, g.d = n, d
        g.amp, g.y_mean, g.y_std = float(meta[0]), float(meta[1]), float(meta[2])
        g.chol_info = 0
        g._score_ws = None
        return g

    # -- views of device state (tests / diagnostics) --------------------------
    def _state_view(self, addr, count):
        base = self._ws.data_ptr()
        off = addr - base
        assert off % 8 == 0 and 0 <= off and off + count * 8 <= self._ws.numel()
        return self._ws[off:off + count * 8].view(torch.float64)

    def L_factor(self):
        return self._state_view(self.model.L, self.n * self.n).view(self.n, self.n)

    def L_inverse(self):
        return self._state_view(self.model.W, self.n * self.n).view(self.n, self.n)

    def alpha(self):
        return self._state_view(self.model.alpha, self.n)

    # -- scoring ---------------------------------------------------------------
    def _ensure_ws(self, m, k):
        need = lib().mpo_gp_score_ws_bytes(ctypes.byref(self.model), int(m), int(k))
        if need == 0:
            raise _lib.MpoError("mpo_gp_score_ws_bytes rejected the shape")
        if self._score_ws is None or self._score_ws.numel() < need:
            self._score_ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._score_ws, need

    def as_candidates(self, cand):
        if isinstance(cand, torch.Tensor):
            t = cand.to(device=self.device, dtype=torch.float64)
        else:
            t = torch.from_numpy(np.ascontiguousarray(np.asarray(cand, dtype=np.float64))).to(self.device)
        t = t.contiguous()
        if t.ndim != 2 or t.shape[1] != self.d:
            raise ValueError(f"candidates must be (m, {self.d}), got {tuple(t.shape)}")
        return t

    def score(self, cand, y_opt, acqs=("EI",), xi=0.01, kappa=1.96, k=0, want_mu_sd=True,
              want_values=True):
        """Score candidates.  Returns a dict with device tensors:
        ``mu``, ``sd`` (m,), ``values`` {acq: (m,)} (the value skopt minimises),
        ``topk`` {acq: (idx int64 (k,), val (k,))}."""
        c = self.as_candidates(cand)
        m = c.shape[0]
        flags = 0
        for a in acqs:
            flags |= _lib.ACQ_FLAGS[a]
        ws, wsb = self._ensure_ws(m, k)
        dev = self.device
        mu = torch.empty(m, dtype=torch.float64, device=dev) if want_mu_sd else None
        sd = torch.empty(m, dtype=torch.float64, device=dev) if want_mu_sd else None
        vals = torch.empty(3, m, dtype=torch.float64, device=dev) if want_values else None
        tki = torch.empty(3, max(k, 1), dtype=torch.int64, device=dev)
        tkv = torch.empty(3, max(k, 1), dtype=torch.float64, device=dev)
        with torch.cuda.device(dev):
            s = _lib.stream_handle(dev)
            check(lib().mpo_gp_acq_score(ctypes.byref(self.model), ptr(c), m, float(y_opt), float(xi),
                                         float(kappa), flags, ptr(mu), ptr(sd), ptr(vals), int(k),
                                         ptr(tki) if k else None, ptr(tkv) if k else None,
                                         ptr(ws), wsb, s), "mpo_gp_acq_score")
        out = {"mu": mu, "sd": sd, "values": {}, "topk": {}}
        for a in acqs:
            r = _lib.ACQ_ROW[a]
            if vals is not None:
                out["values"][a] = vals[r]
            if k:
                out["topk"][a] = (tki[r, :k], tkv[r, :k])
        return out

    def ei_argmax(self, cand, y_opt, xi=0.01):
        """``mpo_gp_ei_score``: (mu, sd, ei=+EI, argmax) on device."""
        c = self.as_candidates(cand)
        m = c.shape[0]
        ws, wsb = self._ensure_ws(m, 1)
        dev = self.device
        mu = torch.empty(m, dtype=torch.float64, device=dev)
        sd = torch.empty(m, dtype=torch.float64, device=dev)
        ei = torch.empty(m, dtype=torch.float64, device=dev)
        am = torch.empty(1, dtype=torch.int64, device=dev)
        with torch.cuda.device(dev):
            check(lib().mpo_gp_ei_score(ctypes.byref(self.model), ptr(c), m, float(y_opt), float(xi), ptr(mu),
                                        ptr(sd), ptr(ei), ptr(am), ptr(ws), wsb, _lib.stream_handle(dev)),
                  "mpo_gp_ei_score")
        return mu, sd, ei, am

    def _ensure_ag(self, B):
        """Pinned host buffers of one polish round (x, acquisition codes, f, g) for B points."""
        if getattr(self, "_ag_cap", 0) < B:
            cap = max(16, B)
            d = self.d
            self._ag_x = torch.empty(cap * d, dtype=torch.float64).pin_memory()
            self._ag_a = torch.empty(cap, dtype=torch.int32).pin_memory()
            self._ag_f = torch.empty(cap, dtype=torch.float64).pin_memory()
            self._ag_g = torch.empty(cap * d, dtype=torch.float64).pin_memory()
            self._ag_np = (self._ag_x.numpy(), self._ag_a.numpy(), self._ag_f.numpy(), self._ag_g.numpy())
            self._ag_ptrs = (self._ag_x.data_ptr(), self._ag_a.data_ptr(), self._ag_f.data_ptr(),
                             self._ag_g.data_ptr())
            self._ag_stream = _lib.stream_handle(self.device)
            self._ag_cap = cap

    def acq_grad(self, X, acq_codes, y_opt, xi=0.01, kappa=1.96):
        """``mpo_gp_acq_grad_host``: minimised acquisition value and gradient at
        the rows of X (B, d) (transformed space), acquisition ``acq_codes[b]``
        (MPO_ACQ_* flag values).  The kernel reads X and the codes from pinned
        host memory and writes f, g into it (no staging copies: a polish round is
        ~30 us of device time, torch's copies and stream context cost as much);
        returns numpy (f (B,), g (B, d))."""
        X = np.asarray(X, dtype=np.float64).reshape(-1, self.d)
        B, d = X.shape
        self._ensure_ag(B)
        xn, an, fn, gn = self._ag_np
        xn[:B * d] = X.reshape(-1)
        an[:B] = acq_codes
        xp, ap, fp, gp = self._ag_ptrs
        rc = lib().mpo_gp_acq_grad_host(ctypes.byref(self.model), xp, B, ap, float(y_opt), float(xi), float(kappa),
                                        fp, gp, self._ag_stream)
        if rc != 0:
            check(rc, "mpo_gp_acq_grad_host")
        return fn[:B].copy(), gn[:B * d].reshape(B, d).copy()

    def polish(self, starts, acq_codes, y_opt, xi, kappa, bounds, ftol, maxiter=20, gtol=1e-5, maxfun=15000):
        """skopt's polish of its best candidates, whole, in ``mpo_gp_polish_host``:
        L-BFGS-B (libmpo.so's host driver) from each row of ``starts`` (B, d) on
        acquisition ``acq_codes[r]``, one ``mpo_gp_acq_grad_host`` round per
        iteration of all live runs.  Returns [(x, f)] per run."""
        starts = np.ascontiguousarray(np.asarray(starts, dtype=np.float64))
        B, d = starts.shape
        if d != self.d:
            raise ValueError(f"polish starts must be (B, {self.d}), got {starts.shape}")
        self._ensure_ag(B)
        codes = np.ascontiguousarray(np.asarray(acq_codes, dtype=np.int32))
        b = np.ascontiguousarray(np.asarray(bounds, dtype=np.float64).reshape(d, 2))
        opts = _lib.MpoLbfgsbOptions(ftol, gtol, maxiter, maxfun, 10, 20)
        x = np.empty((B, d))
        f = np.empty(B)
        stats = np.empty((B, 4), np.int32)
        rounds = ctypes.c_int32(0)
        xp, ap, fp, gp = self._ag_ptrs
        rc = lib().mpo_gp_polish_host(ctypes.byref(self.model), starts.ctypes.data, codes.ctypes.data, B,
                                      b.ctypes.data, ctypes.byref(opts), float(y_opt), float(xi), float(kappa),
                                      xp, ap, fp, gp, x.ctypes.data, f.ctypes.data, stats.ctypes.data,
                                      ctypes.byref(rounds), self._ag_stream)
        if rc != 0:
            check(rc, "mpo_gp_polish_host")
        return [(x[r], float(f[r])) for r in range(B)]

    def predict(self, Xc, return_std=True):
        """skopt ``predict(X, return_std=True)`` -> numpy (mu, sd)."""
        out = self.score(Xc, y_opt=0.0, acqs=("EI",), k=0, want_mu_sd=True, want_values=False)
        mu = out["mu"].cpu().numpy()
        sd = out["sd"].cpu().numpy()
        return (mu, sd) if return_std else mu


def _view_int32(addr, ws, device):
    off = addr - ws.data_ptr()
    return ws[off:off + 4].view(torch.int32)
