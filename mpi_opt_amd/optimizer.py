"""Bayesian optimizer with the ``skopt.Optimizer`` interface the reference drives.

The reference constructs ``skopt.Optimizer(dimensions=..., random_state=13579)``
(/root/reference/coordinator.py:33) and calls ``ask(n)`` (:49), ``tell(X, Y)``
(:69) and pickles it (:52-61); threaded_skopt.py:162-171 shows the same class
with explicit ``base_estimator``/``acq_func``/``acq_optimizer``.  scikit-optimize
is un-vendored and unpinned; its published ``Optimizer`` algorithm is restated:

* ``n_initial_points`` (10) random points, then a GP surrogate
  ``C(1,(0.01,1000)) * Matern(ones(D),(0.01,100),nu=2.5) + White``,
  ``normalize_y=True``, ``n_restarts_optimizer=2`` (``cook_estimator("GP")``);
* acquisition ``gp_hedge`` over {EI, LCB, PI} (xi=0.01, kappa=1.96), each
  scored on ``n_points=10000`` random candidates, the best
  ``n_restarts_optimizer=5`` polished with L-BFGS-B (maxiter 20) -- the
  ``acq_optimizer="auto"`` -> ``"lbfgs"`` path -- and one of the three picked by
  softmax(gains) (``eta=1``) with a multinomial draw;
* ``ask(n, strategy="cl_min")`` = constant-liar batch through a copy.

MI355X mapping: the candidate scoring (posterior + EI/PI/LCB + top-k over the
candidate batch) runs in ``libmpo.so`` on the GPU (:class:`~mpi_opt_amd.gp.DeviceGP`),
together with the GP factorisation, and so does the objective of the GP
hyper-parameter refit (:mod:`~mpi_opt_amd.gp_fit`: LML + gradient, all L-BFGS-B
restarts batched into one launch per iteration), and so does the objective of the
acquisition polish (``mpo_gp_acq_grad``: the 3 x 5 L-BFGS-B runs of one ask step
batched into one launch per iteration).  Only the L-BFGS-B control flow -- the
reference's host-side scipy loop -- stays on the host.
"""
from __future__ import annotations

import copy as _copy
import threading
import time

import numpy as np
from scipy.optimize import fmin_l_bfgs_b

from . import _lib
from .gp_fit import fit_lml
from .space import Space, check_random_state

# --------------------------------------------------------------------------
# GP hyper-parameter fit (device LML objective, sklearn's restart/L-BFGS-B loop)
# --------------------------------------------------------------------------
#: L-BFGS-B driver of the refits and the acquisition polish: "native" (csrc/lbfgsb.cpp,
#: the default: GIL-free, iterates equal to scipy's to rounding) or "scipy" (scipy's own
#: setulb driven from Python: the exact-parity mode, bit for bit scipy's iterates).
DRIVER = "native"


def fit_gp_hyperparameters(Xt, y, random_state=None, n_restarts_optimizer=2, device=None):
    """skopt's GP fit: sklearn GaussianProcessRegressor with the cook_estimator
    kernel + WhiteKernel, normalize_y, L-BFGS-B restarts -- the objective
    (LML + gradient) evaluated by ``mpo_gp_lml_grad``.  Returns (amp, length_scale, noise)."""
    return fit_lml(Xt, y, random_state=random_state, n_restarts_optimizer=n_restarts_optimizer, device=device,
                   driver=DRIVER)


class GPModel:
    """A fitted surrogate: hyper-parameters + its device posterior (rebuilt lazily,
    so the model pickles without device state)."""

    def __init__(self, Xt, y, amp, length_scale, noise, device=None):
        self.Xt = np.asarray(Xt, dtype=float)
        self.y = np.asarray(y, dtype=float)
        self.amp, self.length_scale, self.noise = float(amp), np.asarray(length_scale, float), float(noise)
        self.device = device
        self._dev = None

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_dev"] = None
        return d

    @property
    def dev(self):
        if self._dev is None:
            from .gp import DeviceGP

            self._dev = DeviceGP(self.Xt, self.y, self.amp, self.length_scale, self.noise, device=self.device)
        return self._dev

    def predict_mean(self, X):
        mu, _ = self.dev.predict(np.atleast_2d(X))
        return mu


def polish_lockstep(model, starts, acqs, y_opt, xi, kappa, bounds, maxiter=20, driver="native"):
    """skopt's acquisition polish: ``fmin_l_bfgs_b(gaussian_acquisition_1D, x0,
    bounds, approx_grad=False, maxiter=20)`` from every start ``starts[w]`` of
    acquisition ``acqs[w]``.  The runs are independent; they step in lockstep so
    that each round of evaluations is one ``mpo_gp_acq_grad`` launch over all live
    runs.  ``driver="native"``: the whole polish in ``mpo_gp_polish_host`` (the host
    L-BFGS-B of libmpo.so, no GIL held); "scipy": scipy's setulb driven from
    Python.  Returns [(x, f)] per run."""
    from .gp_fit import FMIN_FTOL, _Lockstep, _setulb, lbfgsb_batched

    codes = np.array([_lib.ACQ_FLAGS[a] for a in acqs], dtype=np.int32)
    if driver == "native":
        return model.dev.polish(np.array(starts), codes, y_opt, xi, kappa, bounds, ftol=FMIN_FTOL, maxiter=maxiter)
    if driver != "scipy":
        raise ValueError(f"driver {driver!r}: 'native' or 'scipy'")

    def evaluate(X, ids):
        return model.dev.acq_grad(X, codes[ids], y_opt, xi, kappa)

    if _setulb() is not None:        # one thread drives every run (setulb reverse communication)
        out, _ = lbfgsb_batched(evaluate, starts, bounds, ftol=FMIN_FTOL, maxiter=maxiter)
        return out

    step = _Lockstep(evaluate, len(starts), pass_ids=True)
    out = [None] * len(starts)
    errors = []

    def run(w):
        try:
            xr, fr, _ = fmin_l_bfgs_b(lambda v: step(w, v), starts[w], bounds=bounds, approx_grad=False,
                                      maxiter=maxiter)
            out[w] = (xr, float(fr))
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
    return out


#: process-wide accounts of the GP work (bench / search reports): refits, their
#: observation counts and the seconds spent refitting vs proposing.  Chains run
#: on worker threads (:mod:`~mpi_opt_amd.chains`), so updates take ``STATS_LOCK``;
#: the seconds are then summed over concurrent workers (device-thread seconds).
STATS = {"refits": 0, "n_sum": 0, "n_max": 0, "refit_s": 0.0, "propose_s": 0.0, "prepare_s": 0.0, "score_s": 0.0,
         "polish_s": 0.0, "samples": []}
STATS_LOCK = threading.Lock()


def reset_stats():
    with STATS_LOCK:
        STATS.update(refits=0, n_sum=0, n_max=0, refit_s=0.0, propose_s=0.0, prepare_s=0.0, score_s=0.0,
                     polish_s=0.0, samples=[])


def merge_stats(delta):
    """Add another process's STATS (a chain worker rank's) into this one's."""
    with STATS_LOCK:
        for k, v in delta.items():
            if k == "n_max":
                STATS[k] = max(STATS[k], v)
            elif k == "samples":
                STATS[k].extend(v)
            else:
                STATS[k] += v


def _record_refit(n, t_refit, t_prepare, t_score, t_polish, t_propose, t_total):
    with STATS_LOCK:
        STATS["refits"] += 1
        STATS["n_sum"] += n
        STATS["n_max"] = max(STATS["n_max"], n)
        STATS["refit_s"] += t_refit
        STATS["prepare_s"] += t_prepare
        STATS["score_s"] += t_score
        STATS["polish_s"] += t_polish
        STATS["propose_s"] += t_propose
        STATS["samples"].append((n, t_total))      # (n, seconds of refit + proposal)


STRATEGIES = ("cl_min", "cl_mean", "cl_max")


class ChainJob:
    """Everything one ``ask(n_points, strategy)`` batch depends on: the optimizer's
    state when ``ask`` was called (its told points, gp_hedge gains, initial-point
    budget and configuration) and the seed the copy draws from the optimizer's
    RandomState.  The batch is a pure function of this record -- the copy never
    touches the asking optimizer again (skopt's ``ask``: ``opt = self.copy(
    random_state=self.rng.randint(...))``, then lies told to ``opt`` only) -- so a
    job can run later, on another thread, stream, process or GPU, and give the
    same points.  Picklable (no device state)."""

    __slots__ = ("config", "Xi", "yi", "gains", "initial_samples", "n_initial_points", "seed", "n_points",
                 "strategy", "trace", "cost")

    def __init__(self, opt, seed, n_points, strategy):
        self.config = opt._config()
        self.Xi = [list(x) for x in opt.Xi]
        self.yi = list(opt.yi)
        self.gains = np.copy(opt.gains_) if hasattr(opt, "gains_") else None
        self.initial_samples = opt._initial_samples
        self.n_initial_points = opt.n_initial_points_
        # an int from ask(); copy(random_state=...) may pass anything check_random_state takes
        self.seed = int(seed) if isinstance(seed, (int, np.integer)) else seed
        self.n_points, self.strategy = int(n_points), strategy
        self.trace = opt.trace is not None
        # LPT weight: a refit costs ~n^2 at these sizes (the LML's n^3 work is spread
        # over n/16 workgroups); one refit per lie once the initial points are spent
        n0 = len(self.yi)
        self.cost = float(sum((n0 + i + 1) ** 2 for i in range(self.n_points)))

    # ---- fixed-layout form for the tensor collectives (blocks.DistributedEvaluator) ----
    META = 10   # int64 words per job: n, D, has_gains, n_initial_points, seed, n_points, strategy, trace, n_init, blob

    def encode(self):
        """(meta int64 [META], blob f64): the job without its config (sent once per
        search).  Points cross as (value, type code) pairs (collectives.encode_points)."""
        from .collectives import encode_points

        if not isinstance(self.seed, (int, np.integer)):
            raise TypeError("ChainJob.encode: the copy's seed must be an int")
        if self.trace:
            raise NotImplementedError("ChainJob.encode: refit traces (parity tests) do not cross ranks")
        n = len(self.yi)
        xv, xc = encode_points(self.Xi) if n else (np.zeros((0, 0)), np.zeros((0, 0)))
        d = xv.shape[1] if n else 0
        parts = [xv.ravel(), xc.ravel(), np.asarray(self.yi, dtype=np.float64)]
        if self.gains is not None:
            parts.append(np.asarray(self.gains, dtype=np.float64).ravel())
        n_init = -1
        if self.initial_samples is not None:
            iv, ic = encode_points([list(x) for x in self.initial_samples])
            n_init = len(iv)
            d = d or iv.shape[1]
            parts += [iv.ravel(), ic.ravel()]
        blob = np.concatenate(parts) if parts else np.zeros(0)
        meta = np.array([n, d, -1 if self.gains is None else len(np.ravel(self.gains)), int(self.n_initial_points),
                         int(self.seed), self.n_points, STRATEGIES.index(self.strategy), 0, n_init, len(blob)],
                        dtype=np.int64)
        return meta, blob

    @classmethod
    def decode(cls, meta, blob, config):
        """Inverse of :meth:`encode` with the search's ``config``."""
        from .collectives import decode_points

        n, d, ng, nip, seed, npts, strat, _trace, n_init, _ = (int(v) for v in meta)
        job = cls.__new__(cls)
        o = 0
        xv = blob[o:o + n * d].reshape(n, d); o += n * d
        xc = blob[o:o + n * d].reshape(n, d); o += n * d
        job.Xi = decode_points(xv, xc)
        job.yi = [float(v) for v in blob[o:o + n]]; o += n
        job.gains = None
        if ng >= 0:
            job.gains = np.array(blob[o:o + ng], dtype=np.float64); o += ng
        job.initial_samples = None
        if n_init >= 0:
            iv = blob[o:o + n_init * d].reshape(n_init, d); o += n_init * d
            ic = blob[o:o + n_init * d].reshape(n_init, d); o += n_init * d
            job.initial_samples = decode_points(iv, ic)
        job.config = config
        job.n_initial_points = nip
        job.seed = seed
        job.n_points, job.strategy, job.trace = npts, STRATEGIES[strat], False
        job.cost = float(sum((n + i + 1) ** 2 for i in range(npts)))
        return job

    def copy_optimizer(self, device=None, scorer=None):
        """``Optimizer.copy(random_state=seed)`` of the asking optimizer, on ``device``."""
        opt = Optimizer(random_state=self.seed, device=device, scorer=scorer, **self.config)
        opt._initial_samples = self.initial_samples
        if self.gains is not None:
            opt.gains_ = np.copy(self.gains)
        opt.trace = [] if self.trace else None
        if self.Xi:
            opt._tell([list(x) for x in self.Xi], list(self.yi))
        return opt

    def run(self, device=None, scorer=None):
        """The batch: (list of points, the copy's refit trace or None)."""
        opt = self.copy_optimizer(device, scorer)
        return _lie_loop(opt, self.n_points, self.strategy), opt.trace


def _lie_loop(opt, n_points, strategy):
    """skopt's constant-liar loop on the copy ``opt``: ask, then tell the lie."""
    X = []
    for _ in range(n_points):
        x = opt._ask()
        X.append(x)
        if strategy == "cl_min":
            lie = np.min(opt.yi) if opt.yi else 0.0
        elif strategy == "cl_mean":
            lie = np.mean(opt.yi) if opt.yi else 0.0
        else:
            lie = np.max(opt.yi) if opt.yi else 0.0
        opt._tell(x, lie)
        # only the newest surrogate is used again (gains, the next proposal):
        # release the older ones' device factorisations as the chain grows
        for m in opt.models[:-1]:
            m._dev = None
    return X


class OptimizeResult(dict):
    __getattr__ = dict.get

    def __setattr__(self, k, v):
        self[k] = v


class Optimizer:
    """Drop-in for ``skopt.Optimizer`` (GP base estimator, device acquisition).

    ``acq_optimizer_kwargs["n_restarts_optimizer"]`` (default 5) may exceed the
    device top-k width (``MPO_TOPK_MAX`` = 8); the acquisition rows are then
    sorted whole on the device instead."""

    def __init__(self, dimensions, base_estimator="gp", n_random_starts=None, n_initial_points=10,
                 initial_point_generator="random", acq_func="gp_hedge", acq_optimizer="auto",
                 random_state=None, model_queue_size=None, acq_func_kwargs=None, acq_optimizer_kwargs=None,
                 device=None, _gp_seed=None, scorer=None, chain_executor=None):
        self.rng = check_random_state(random_state)
        self.space = Space(dimensions)
        if n_random_starts is not None:
            n_initial_points = n_random_starts
        if isinstance(base_estimator, str):
            base_estimator = base_estimator.lower()
        if base_estimator not in ("gp", "dummy"):
            raise ValueError(f"base_estimator {base_estimator!r}: this build supports 'gp' and 'dummy'")
        self.base_estimator_ = base_estimator
        # skopt cooks the estimator once, with random_state=rng.randint(...); a copy()
        # receives the cooked estimator (no draw), and every refit clones it, so the
        # GP restarts draw from the same seed at every fit.
        self._gp_seed = self.rng.randint(0, np.iinfo(np.int32).max) if _gp_seed is None else _gp_seed
        if acq_func not in ("gp_hedge", "EI", "PI", "LCB"):
            raise ValueError(f"acq_func {acq_func!r} not supported")
        self.acq_func = acq_func
        self.acq_func_kwargs = dict(acq_func_kwargs or {})
        self.eta = self.acq_func_kwargs.get("eta", 1.0)
        if acq_optimizer == "auto":
            acq_optimizer = "lbfgs"
        if acq_optimizer not in ("lbfgs", "sampling"):
            raise ValueError(f"acq_optimizer {acq_optimizer!r} not supported")
        self.acq_optimizer = acq_optimizer
        self.acq_optimizer_kwargs = dict(acq_optimizer_kwargs or {})
        self.n_points = self.acq_optimizer_kwargs.get("n_points", 10000)
        self.n_restarts_optimizer = self.acq_optimizer_kwargs.get("n_restarts_optimizer", 5)
        self.n_initial_points_ = n_initial_points
        self._n_initial_points = n_initial_points
        self._initial_point_generator = initial_point_generator
        self._initial_samples = None
        self.model_queue_size = model_queue_size
        self.device = device
        self.scorer = scorer
        self.cand_acq_funcs_ = ["EI", "LCB", "PI"] if acq_func == "gp_hedge" else [acq_func]
        if acq_func == "gp_hedge":
            self.gains_ = np.zeros(3)
        self.Xi, self.yi, self.models = [], [], []
        self.cache_ = {}
        self.trace = None       # a list here records each refit (theta, top-k, polish, pick) for parity tests
        # optional: runs ask(n) batches asynchronously (mpi_opt_amd.chains); ask then
        # returns a LazyBatch whose points resolve when first used
        self.chain_executor = chain_executor

    def __setstate__(self, d):
        # checkpoints written before these attributes existed resume with their defaults
        d.setdefault("trace", None)
        d.setdefault("chain_executor", None)
        self.__dict__.update(d)

    def _config(self):
        """The constructor arguments a copy() shares with this optimizer."""
        return dict(dimensions=self.space.dimensions, base_estimator=self.base_estimator_,
                    n_initial_points=self.n_initial_points_, initial_point_generator=self._initial_point_generator,
                    acq_func=self.acq_func, acq_optimizer=self.acq_optimizer, acq_func_kwargs=self.acq_func_kwargs,
                    acq_optimizer_kwargs=self.acq_optimizer_kwargs, _gp_seed=self._gp_seed)

    # ---- ask -------------------------------------------------------------------
    def copy(self, random_state=None):
        return ChainJob(self, random_state, 0, "cl_min").copy_optimizer(self.device, self.scorer)

    def ask(self, n_points=None, strategy="cl_min"):
        if n_points is None:
            return self._ask()
        if strategy not in ("cl_min", "cl_mean", "cl_max"):
            raise ValueError(f"strategy {strategy!r}")
        if (n_points, strategy) in self.cache_:
            return self.cache_[(n_points, strategy)]
        job = ChainJob(self, self.rng.randint(0, np.iinfo(np.int32).max), n_points, strategy)
        if self.chain_executor is not None:
            X = self.chain_executor.submit(job)
        else:
            X, trace = job.run(self.device, self.scorer)
            if trace is not None:
                self.batch_trace = trace
        self.cache_ = {(n_points, strategy): X}
        return X

    def _ask(self):
        if self._n_initial_points > 0 or self.base_estimator_ == "dummy":
            if self._initial_samples is None:
                return self.space.rvs(random_state=self.rng)[0]
            return self._initial_samples[len(self._initial_samples) - self._n_initial_points]
        if not self.models:
            raise RuntimeError("Random evaluations exhausted and no model has been fit.")
        return self._next_x

    # ---- tell ------------------------------------------------------------------
    def tell(self, x, y, fit=True):
        from .chains import LazyPoint, resolve

        if isinstance(x, LazyPoint):         # points popped from a lazy ask batch
            x = resolve(x)
        elif len(x) and isinstance(x[0], LazyPoint):
            x = [resolve(v) for v in x]
        if len(x) and isinstance(x[0], (list, tuple, np.ndarray)):
            if not np.ndim(y) == 1 or len(y) != len(x):
                raise ValueError("tell: X and y must have matching lengths")
        return self._tell(x, y, fit=fit)

    def _tell(self, x, y, fit=True):
        if len(x) and isinstance(x[0], (list, tuple, np.ndarray)):
            self.Xi.extend([list(v) for v in x])
            self.yi.extend([float(v) for v in y])
            self._n_initial_points -= len(y)
        else:
            self.Xi.append(list(x))
            self.yi.append(float(y))
            self._n_initial_points -= 1
        self.cache_ = {}
        if fit and self._n_initial_points <= 0 and self.base_estimator_ == "gp":
            self._fit_and_propose()
        return self._result()

    def _fit_and_propose(self):
        Xt = self.space.transform(self.Xi)
        y = np.asarray(self.yi, dtype=float)
        t0 = time.perf_counter()
        amp, ls, noise = fit_gp_hyperparameters(Xt, y, random_state=self._gp_seed, device=self.device)
        t1 = time.perf_counter()
        est = GPModel(Xt, y, amp, ls, noise, device=self.device)
        est.dev                                   # the device posterior (mpo_gp_prepare)
        t2 = time.perf_counter()
        if hasattr(self, "next_xs_") and self.acq_func == "gp_hedge":
            self.gains_ -= est.predict_mean(np.vstack(self.next_xs_))
        if self.model_queue_size is None or self.model_queue_size > 0:
            self.models.append(est)
            if self.model_queue_size is not None and len(self.models) > self.model_queue_size:
                self.models.pop(0)

        X = self.space.rvs_transformed(n_samples=self.n_points, random_state=self.rng)
        y_opt = float(np.min(self.yi))
        xi = self.acq_func_kwargs.get("xi", 0.01)
        kappa = self.acq_func_kwargs.get("kappa", 1.96)
        k = 1 if self.acq_optimizer == "sampling" else min(self.n_restarts_optimizer, X.shape[0])
        t3 = time.perf_counter()
        top = self._score_topk(est, X, y_opt, xi, kappa, k)
        t4 = time.perf_counter()
        t_polish = 0.0
        rec = {"theta": (est.amp, est.length_scale.copy(), est.noise), "top": dict(top), "polished": {}} \
            if self.trace is not None else None
        self.next_xs_ = []
        if self.acq_optimizer == "lbfgs":
            runs = [(a, i) for a in self.cand_acq_funcs_ for i in top[a]]
            polished = polish_lockstep(est, [X[i] for _, i in runs], [a for a, _ in runs], y_opt, xi, kappa,
                                       self.space.transformed_bounds, driver=DRIVER)
            t_polish = time.perf_counter() - t4
        for acq in self.cand_acq_funcs_:
            idx = top[acq]
            if self.acq_optimizer == "sampling":
                next_x = X[idx[0]]
            else:
                results = [polished[w] for w, (a, _) in enumerate(runs) if a == acq]
                cand_xs = np.array([r[0] for r in results])
                cand_acqs = np.array([r[1] for r in results])
                next_x = cand_xs[np.argmin(cand_acqs)]
                if rec is not None:
                    rec["polished"][acq] = (cand_xs, cand_acqs)
            self.next_xs_.append(np.clip(next_x, 0.0, 1.0))
        if self.acq_func == "gp_hedge":
            logits = np.array(self.gains_) - np.max(self.gains_)
            probs = np.exp(self.eta * logits)
            probs /= probs.sum()
            pick = int(np.argmax(self.rng.multinomial(1, probs)))
        else:
            pick = 0
        next_x = self.next_xs_[pick]
        if rec is not None:
            rec["pick"] = pick
            rec["gains"] = np.copy(getattr(self, "gains_", np.zeros(0)))
            self.trace.append(rec)
        self._next_x = self.space.inverse_transform(next_x.reshape(1, -1))[0]
        t5 = time.perf_counter()
        _record_refit(len(y), t1 - t0, t2 - t1, t4 - t3, t_polish, t5 - t1, t5 - t0)

    def _score_topk(self, est, X, y_opt, xi, kappa, k):
        """skopt's ``np.argsort(values)[:k]`` per acquisition (lowest index first on
        ties).  The device top-k holds up to MPO_TOPK_MAX entries; a larger
        ``n_restarts_optimizer`` takes the full value rows and a stable sort.  With
        a ``scorer`` (e.g. blocks.ShardedScorer) the candidates are split over GPUs."""
        acqs = tuple(self.cand_acq_funcs_)
        if self.scorer is not None:
            return self.scorer(est, X, y_opt, acqs, xi, kappa, k)
        from .blocks import _device_topk

        return {a: idx for a, (vals, idx) in _device_topk(est, X, y_opt, acqs, xi, kappa, k).items()}

    def _result(self):
        if not self.yi:
            return OptimizeResult(x=None, fun=None, x_iters=[], func_vals=np.array([]), models=self.models,
                                  space=self.space)
        best = int(np.argmin(self.yi))
        return OptimizeResult(x=list(self.Xi[best]), fun=float(self.yi[best]), x_iters=list(self.Xi),
                              func_vals=np.asarray(self.yi), models=self.models, space=self.space,
                              random_state=self.rng)

    def run(self, func, n_iter=1):
        for _ in range(n_iter):
            x = self.ask()
            self.tell(x, func(x))
        return self._result()

    def set_runtime(self, device=None, scorer=None, chain_executor=None):
        """Re-attach the per-run state a checkpoint does not carry (the device of
        this run, when distributed the candidate scorer, the ask-batch executor);
        the models' device posteriors are rebuilt lazily on ``device``."""
        self.device = device
        self.scorer = scorer
        self.chain_executor = chain_executor
        for m in self.models:
            m.device, m._dev = device, None

    def __getstate__(self):
        d = _copy.copy(self.__dict__)
        d["scorer"] = None          # a process-group handle is not checkpoint state
        d["chain_executor"] = None  # nor are worker threads
        return d
