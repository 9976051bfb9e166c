"""Synthetic inputs of SURVEY §8(d) (no datasets are available offline).

GP/EI: X ~ U[0,1]^{n x d}, y = sin(X w) + 0.1 eps (w, eps ~ N(0,1)), candidates ~
U[0,1]^{m x d} -- legacy numpy RandomState streams, so the same seeds give the
same arrays everywhere (tests/test_synthetic.py pins them to the oracle's copy).
"""
import numpy as np


def gp_problem(n=200, d=10, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.uniform(size=(n, d))
    w = rng.randn(d)
    y = np.sin(X @ w) + 0.1 * rng.randn(n)
    return X, y


def gp_candidates(m, d=10, seed=1):
    return np.random.RandomState(seed).uniform(size=(m, d))
