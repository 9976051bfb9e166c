"""Generate the GP/EI golden fixtures ``tests/golden/gp_ei_*.npz``.

Run from the repo root:  ``python tests/golden/make_gp_golden.py``

Each fixture is data only (inputs + expected outputs):

* inputs: observations ``X`` (transformed, [0,1]^D), raw ``y``, candidates ``C``,
  ``xi``, ``kappa``;
* sklearn 1.7.2 outputs (the arithmetic base skopt subclasses, present here):
  fitted hyper-parameters (``amp``, ``ls``, ``noise``), ``L_``, ``alpha_``,
  and ``predict(C, return_std=True)`` with the WhiteKernel noise zeroed the way
  skopt does after ``fit`` (``sk_mu``, ``sk_sd``);
* oracle outputs: skopt einsum-form ``mu``/``sd``; 80-bit ``mu_exact``/``sd_exact``;
  minimised acquisition values ``v_EI``/``v_PI``/``v_LCB``; ``argmin_*``;
  ``top5_*``; the EI top-2 relative gap (how far the argmax is from a tie).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import gp_ei as O  # noqa: E402

CASES = [
    # name, n_obs, dims, n_candidates, seed
    ("n200_d10", 200, 10, 4096, 0),   # BASELINE configs[1] shape (candidate subset)
    ("n12_d5", 12, 5, 1000, 3),       # mnist space right after n_initial_points=10
    ("n57_d3", 57, 3, 777, 5),        # ragged: N, D, M not multiples of any tile
]


def make(name, n, d, m, seed):
    X, y = O.synthetic_problem(n, d, seed)
    C = O.synthetic_candidates(m, d, seed + 1)
    st, gpr = O.fit_skopt_gp(X, y, random_state=seed)
    gpr.kernel_.set_params(k2__noise_level=0.0)   # skopt's post-fit white zeroing
    sk_mu, sk_sd = gpr.predict(C, return_std=True)
    mu, sd = O.posterior_skopt(st, C)
    mu_x, sd_x = O.posterior_exact(st, C)
    y_opt = float(np.min(y))
    out = dict(X=X, y=y, C=C, xi=0.01, kappa=1.96, y_opt=y_opt,
               amp=st.amp, ls=st.length_scale, noise=st.noise,
               y_mean=st.y_mean, y_std=st.y_std,
               sk_L=gpr.L_, sk_alpha=gpr.alpha_, sk_mu=sk_mu, sk_sd=sk_sd,
               mu=mu, sd=sd, mu_exact=mu_x.astype(np.float64), sd_exact=sd_x.astype(np.float64),
               qbound=O.quad_form_abs_bound(st, C))
    for acq in ("EI", "PI", "LCB"):
        v = O.acquisition_values(mu, sd, y_opt, acq)
        out["v_" + acq] = v
        out["argmin_" + acq] = O.argmin_lowest(v)
        out["top5_" + acq] = O.topk_lowest(v, 5)
    ei = -out["v_EI"]
    srt = np.sort(ei)[::-1]
    out["ei_top2_relgap"] = float((srt[0] - srt[1]) / abs(srt[0]))
    path = os.path.join(HERE, f"gp_ei_{name}.npz")
    np.savez_compressed(path, **out)
    print(path, "theta amp=%.4g noise=%.3g" % (st.amp, st.noise),
          "argmax EI", out["argmin_EI"], "gap %.3g" % out["ei_top2_relgap"])


if __name__ == "__main__":
    for c in CASES:
        make(*c)
