import numpy as np

from mpi_opt_amd import synthetic
from oracle import gp_ei as O


def test_synthetic_recipes_match_the_oracle():
    X, y = synthetic.gp_problem(50, 4, 3)
    Xo, yo = O.synthetic_problem(50, 4, 3)
    assert np.array_equal(X, Xo) and np.array_equal(y, yo)
    assert np.array_equal(synthetic.gp_candidates(99, 4, 5), O.synthetic_candidates(99, 4, 5))
