"""Generate ``tests/golden/gp_lml.npz``: LML + gradient and the fitted theta of
skopt's GP refit, from scikit-learn 1.7.2 itself (the arithmetic base skopt
subclasses; present in this container).

Run from the repo root:  ``python tests/golden/make_lml_golden.py``

Data only: for each case (name, n, d, seed) the inputs ``X``/``y`` come from the
oracle's synthetic recipe; the thetas are the kernel start, the sklearn optimum,
two uniform draws inside the bounds and two corners of the bounds; the outputs
are ``GaussianProcessRegressor.log_marginal_likelihood(theta, eval_gradient=True)``
and the fitted ``kernel_.theta`` / ``log_marginal_likelihood_value_``.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import gp_ei as O  # noqa: E402

CASES = [("n200_d10", 200, 10, 0), ("n12_d5", 12, 5, 3), ("n57_d3", 57, 3, 5), ("n230_d4", 230, 4, 7), ("n130_d6", 130, 6, 11),
         ("n256_d10", 256, 10, 13), ("n500_d10", 500, 10, 17)]


def main():
    out = {}
    for name, n, d, seed in CASES:
        X, y = O.synthetic_problem(n, d, seed)
        st, gpr = O.fit_skopt_gp(X, y, random_state=seed)
        b = gpr.kernel_.bounds
        rng = np.random.RandomState(100 + seed)
        thetas = [np.zeros(d + 2), gpr.kernel_.theta.copy(),
                  rng.uniform(b[:, 0], b[:, 1]), rng.uniform(b[:, 0], b[:, 1]),
                  np.r_[b[0, 1], b[1:d + 1, 0], b[d + 1, 0]],          # amp max, ls min, noise min
                  np.r_[b[0, 0], b[1:d + 1, 1], b[d + 1, 1]]]          # amp min, ls max, noise max
        T = np.stack(thetas)
        L, G = zip(*[gpr.log_marginal_likelihood(t, eval_gradient=True) for t in T])
        out[name + "_X"], out[name + "_y"], out[name + "_theta"] = X, y, T
        out[name + "_lml"], out[name + "_grad"] = np.array(L), np.stack(G)
        out[name + "_fit_theta"] = gpr.kernel_.theta.copy()
        out[name + "_fit_lml"] = np.float64(gpr.log_marginal_likelihood_value_)
        out[name + "_seed"] = np.int64(seed)
        print(name, "fit lml %.6f" % gpr.log_marginal_likelihood_value_, np.exp(gpr.kernel_.theta[[0, -1]]))
    np.savez_compressed(os.path.join(HERE, "gp_lml.npz"), **out)


if __name__ == "__main__":
    main()
