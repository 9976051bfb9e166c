import numpy as np
import pytest

from mpi_opt_amd.space import Categorical, Integer, Real, Space, check_dimension


def test_dimension_inference():
    assert isinstance(check_dimension((1, 6)), Integer)
    assert isinstance(check_dimension((0.0, 1.0)), Real)
    assert isinstance(check_dimension((1, 6.0)), Real)
    assert isinstance(check_dimension(["a", "b", "c"]), Categorical)
    r = check_dimension((1e-5, 1.0, "log-uniform"))
    assert isinstance(r, Real) and r.prior == "log-uniform"


def test_transform_roundtrip_and_bounds():
    sp = Space([Integer(10, 50, name="nb_filters"), Integer(2, 10), Real(0.0, 1.0, name="dropout"),
                Real(1e-4, 1.0, prior="log-uniform"), Categorical([1, 2, 5]), Categorical(["x", "y"])])
    X = sp.rvs(500, random_state=3)
    for x in X:
        assert x in sp
    Xt = sp.transform(X)
    assert Xt.shape == (500, sp.transformed_n_dims) == (500, 8)
    assert Xt.min() >= 0.0 and Xt.max() <= 1.0
    back = sp.inverse_transform(Xt)
    for a, b in zip(X, back):
        assert a[0] == b[0] and a[1] == b[1] and a[4] == b[4] and a[5] == b[5]
        assert abs(a[2] - b[2]) < 1e-12 and abs(a[3] - b[3]) / a[3] < 1e-12


def test_integer_normalize_semantics():
    d = Integer(2, 10)
    assert np.allclose(d.transform([2, 6, 10]), [0.0, 0.5, 1.0])
    assert list(d.inverse_transform([0.0, 0.49, 0.51, 1.0, 1.2])) == [2, 6, 6, 10, 10]


def test_rvs_deterministic_and_covering():
    sp = Space([Integer(2, 10)])
    a = sp.rvs(2000, random_state=1)
    b = sp.rvs(2000, random_state=1)
    assert a == b
    assert {v[0] for v in a} == set(range(2, 11))


def test_bad_dimensions():
    with pytest.raises(ValueError):
        Real(1.0, 0.0)
    with pytest.raises(ValueError):
        check_dimension("nope")


def test_rvs_transformed_is_transform_of_rvs():
    """The candidate sampler draws exactly what transform(rvs()) would, in the same
    random-stream order (the next draw after it agrees too)."""
    from mpi_opt_amd.models import mnist_space
    from mpi_opt_amd.space import Categorical, Integer, Real, Space

    for dims in (mnist_space(), [Real(1e-5, 1e1, prior="log-uniform"), Integer(3, 9), Categorical(["a", "b", "c"]),
                                 Real(-2.0, 3.0), Categorical([True, False])]):
        sp = Space(dims)
        r1, r2 = np.random.RandomState(7), np.random.RandomState(7)
        a = sp.transform(sp.rvs(n_samples=500, random_state=r1))
        b = sp.rvs_transformed(n_samples=500, random_state=r2)
        assert a.shape == b.shape and np.array_equal(a, b)
        assert r1.uniform() == r2.uniform()
