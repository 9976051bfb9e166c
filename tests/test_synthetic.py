import numpy as np

from mpi_opt_amd import synthetic
from oracle import gp_ei as O


def test_synthetic_recipes_match_the_oracle():
    X, y = synthetic.gp_problem(50, 4, 3)
    Xo, yo = O.synthetic_problem(50, 4, 3)
    assert np.array_equal(X, Xo) and np.array_equal(y, yo)
    assert np.array_equal(synthetic.gp_candidates(99, 4, 5), O.synthetic_candidates(99, 4, 5))


def test_trajectory_case_init_matches_product_init():
    """The fixture generator's glorot draw equals the product's (same numpy stream)."""
    import numpy as np

    from mpi_opt_amd.population import TrialSpec, glorot_uniform_init
    from tests import trajectory_cases as T

    for m in T.pop_members()[:7] + T.EPOCH_MEMBERS:
        a = T.glorot_init(*m[:4], m[8])
        b = glorot_uniform_init(TrialSpec(*m[:6], seed=m[7]), m[8])
        assert all(np.array_equal(a[n], b[n]) for n in a)
