"""Search-space dimensions, drop-in for the ``skopt.space`` names the reference uses.

The reference builds its spaces as named ``Real`` / ``Integer`` / ``Categorical``
lists (/root/reference/hyperparameter_search_option3.py:110-114, 126-133, 146-152)
or as bare ``(lo, hi)`` tuples (/root/reference/base_model.py:47-52, 75-83;
OptimizeCNN.py:69-73; hyperparameter_search_option0.py:93-104) that skopt infers.
scikit-optimize is an un-vendored, unpinned dependency; its published behaviour
is restated here for the parts the hot path needs:

* ``transform`` to the GP's unit hypercube (``normalize_dimensions``): Real
  ``(x - lo)/(hi - lo)`` (log10-warped first for ``prior="log-uniform"``),
  Integer ``(round(x) - lo)/(hi - lo)``, Categorical one-hot (a single 0/1
  column for two categories);
* ``inverse_transform`` with clipping, integer rounding, category argmax;
* ``rvs``: each dimension draws ``n`` values in turn from one RandomState
  (uniform in the normalized space, inclusive upper bound, then inverse
  transformed; categories uniformly).
"""
from __future__ import annotations

import numbers

import numpy as np


def check_random_state(seed):
    if seed is None or seed is np.random:
        return np.random.mtrand._rand
    if isinstance(seed, numbers.Integral):
        return np.random.RandomState(seed)
    if isinstance(seed, np.random.RandomState):
        return seed
    raise ValueError(f"{seed!r} cannot be used to seed a RandomState")


def _uniform_inclusive(rng, n):
    # scipy uniform(0, nextafter(1, 2)).rvs: U[0, 1] with the upper bound reachable
    return rng.uniform(0.0, np.nextafter(1.0, 2.0), size=n)


class Dimension:
    name = None

    @property
    def transformed_size(self):
        return 1


class Real(Dimension):
    def __init__(self, low, high, prior="uniform", base=10, transform=None, name=None, dtype=float):
        if high <= low:
            raise ValueError(f"Real: low ({low}) must be < high ({high})")
        if prior not in ("uniform", "log-uniform"):
            raise ValueError(f"Real: unknown prior {prior!r}")
        if prior == "log-uniform" and low <= 0:
            raise ValueError("Real: log-uniform prior needs low > 0")
        self.low, self.high, self.prior, self.base = float(low), float(high), prior, base
        self.name = name
        self.dtype = dtype

    def __repr__(self):
        return f"Real(low={self.low}, high={self.high}, prior='{self.prior}', name={self.name!r})"

    def _warp(self, x):
        x = np.asarray(x, dtype=float)
        if self.prior == "log-uniform":
            return np.log(x) / np.log(self.base), np.log(self.low) / np.log(self.base), \
                np.log(self.high) / np.log(self.base)
        return x, self.low, self.high

    def transform(self, x):
        w, lo, hi = self._warp(x)
        return (w - lo) / (hi - lo)

    def inverse_transform(self, xt):
        xt = np.asarray(xt, dtype=float)
        if self.prior == "log-uniform":
            lo, hi = np.log(self.low) / np.log(self.base), np.log(self.high) / np.log(self.base)
            x = np.power(float(self.base), xt * (hi - lo) + lo)
        else:
            x = xt * (self.high - self.low) + self.low
        return np.clip(x, self.low, self.high)

    def rvs(self, n, rng):
        return self.inverse_transform(_uniform_inclusive(rng, n))

    @property
    def bounds(self):
        return (self.low, self.high)

    def __contains__(self, x):
        return self.low <= x <= self.high

    def __eq__(self, o):
        return isinstance(o, Real) and (self.low, self.high, self.prior, self.name) == (o.low, o.high, o.prior, o.name)


class Integer(Dimension):
    def __init__(self, low, high, prior="uniform", base=10, transform=None, name=None, dtype=np.int64):
        if high < low:
            raise ValueError(f"Integer: low ({low}) must be <= high ({high})")
        self.low, self.high = int(low), int(high)
        self.prior, self.base = prior, base
        self.name = name
        self.dtype = dtype

    def __repr__(self):
        return f"Integer(low={self.low}, high={self.high}, name={self.name!r})"

    def transform(self, x):
        span = self.high - self.low
        if span == 0:
            return np.zeros_like(np.asarray(x, dtype=float))
        return (np.round(np.asarray(x, dtype=float)) - self.low) / span

    def inverse_transform(self, xt):
        x = np.asarray(xt, dtype=float) * (self.high - self.low) + self.low
        return np.clip(np.round(x), self.low, self.high).astype(np.int64)

    def rvs(self, n, rng):
        return self.inverse_transform(_uniform_inclusive(rng, n))

    @property
    def bounds(self):
        return (self.low, self.high)

    def __contains__(self, x):
        return self.low <= x <= self.high

    def __eq__(self, o):
        return isinstance(o, Integer) and (self.low, self.high, self.name) == (o.low, o.high, o.name)


class Categorical(Dimension):
    def __init__(self, categories, prior=None, transform=None, name=None):
        self.categories = tuple(categories)
        if len(self.categories) < 1:
            raise ValueError("Categorical needs at least one category")
        self.name = name
        self.prior = prior

    def __repr__(self):
        return f"Categorical(categories={self.categories}, name={self.name!r})"

    @property
    def transformed_size(self):
        return 1 if len(self.categories) <= 2 else len(self.categories)

    def _index(self, v):
        for i, c in enumerate(self.categories):
            if c == v:
                return i
        raise ValueError(f"{v!r} not in {self.categories}")

    def transform(self, x):
        idx = np.array([self._index(v) for v in np.atleast_1d(x)])
        if self.transformed_size == 1:
            return idx.astype(float)
        out = np.zeros((idx.size, len(self.categories)))
        out[np.arange(idx.size), idx] = 1.0
        return out

    def inverse_transform(self, xt):
        xt = np.asarray(xt, dtype=float)
        if self.transformed_size == 1:
            idx = np.clip(np.round(xt.reshape(-1)), 0, len(self.categories) - 1).astype(int)
        else:
            idx = np.argmax(xt.reshape(-1, len(self.categories)), axis=1)
        return [self.categories[i] for i in idx]

    def rvs(self, n, rng):
        return [self.categories[i] for i in rng.randint(0, len(self.categories), size=n)]

    @property
    def bounds(self):
        return self.categories

    def __contains__(self, x):
        return x in self.categories

    def __eq__(self, o):
        return isinstance(o, Categorical) and (self.categories, self.name) == (o.categories, o.name)


def check_dimension(dim):
    """skopt's inference for tuple / list specifications."""
    if isinstance(dim, Dimension):
        return dim
    if isinstance(dim, list):
        return Categorical(dim)
    if isinstance(dim, tuple):
        if len(dim) == 2 and all(isinstance(v, numbers.Integral) and not isinstance(v, bool) for v in dim):
            return Integer(*dim)
        if len(dim) == 2:
            return Real(*dim)
        if len(dim) == 3 and isinstance(dim[2], str):
            lo, hi, prior = dim
            if isinstance(lo, numbers.Integral) and isinstance(hi, numbers.Integral):
                return Integer(lo, hi, prior=prior)
            return Real(lo, hi, prior=prior)
        return Categorical(list(dim))
    raise ValueError(f"invalid dimension {dim!r}")


class Space:
    def __init__(self, dimensions):
        self.dimensions = [check_dimension(d) for d in dimensions]

    def __len__(self):
        return len(self.dimensions)

    @property
    def n_dims(self):
        return len(self.dimensions)

    @property
    def transformed_n_dims(self):
        return sum(d.transformed_size for d in self.dimensions)

    @property
    def dimension_names(self):
        return [d.name for d in self.dimensions]

    @property
    def is_categorical(self):
        return all(isinstance(d, Categorical) for d in self.dimensions)

    @property
    def bounds(self):
        return [d.bounds for d in self.dimensions]

    @property
    def transformed_bounds(self):
        return [(0.0, 1.0)] * self.transformed_n_dims

    def rvs(self, n_samples=1, random_state=None):
        rng = check_random_state(random_state)
        cols = [d.rvs(n_samples, rng) for d in self.dimensions]
        return [[_py(cols[j][i]) for j in range(len(cols))] for i in range(n_samples)]

    def rvs_transformed(self, n_samples=1, random_state=None):
        """``transform(rvs(n_samples, random_state))`` without the round trip through
        Python lists: the same draws in the same order (skopt draws column by
        column), each column transformed as a numpy array -- the same values.  The
        acquisition candidates of every ask (n_points = 10000) come from here."""
        rng = check_random_state(random_state)
        cols = []
        for d in self.dimensions:
            t = np.asarray(d.transform(d.rvs(n_samples, rng)), dtype=float)
            cols.append(t.reshape(n_samples, -1))
        return np.hstack(cols) if cols else np.zeros((n_samples, 0))

    def transform(self, X):
        X = [list(x) for x in X]
        cols = []
        for j, d in enumerate(self.dimensions):
            t = np.asarray(d.transform([x[j] for x in X]), dtype=float)
            cols.append(t.reshape(len(X), -1))
        return np.hstack(cols) if cols else np.zeros((len(X), 0))

    def inverse_transform(self, Xt):
        Xt = np.atleast_2d(np.asarray(Xt, dtype=float))
        out_cols, c = [], 0
        for d in self.dimensions:
            w = d.transformed_size
            out_cols.append(d.inverse_transform(Xt[:, c:c + w] if w > 1 else Xt[:, c]))
            c += w
        return [[_py(out_cols[j][i]) for j in range(len(out_cols))] for i in range(Xt.shape[0])]

    def distance(self, a, b):
        return float(np.sqrt(np.sum((self.transform([a]) - self.transform([b])) ** 2)))

    def __contains__(self, point):
        return all(v in d for v, d in zip(point, self.dimensions))


def _py(v):
    if isinstance(v, np.integer):
        return int(v)
    if isinstance(v, np.floating):
        return float(v)
    return v
