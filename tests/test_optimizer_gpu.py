"""Optimizer end to end on the device acquisition path."""
import numpy as np
import pytest

from oracle import gp_ei as O

pytestmark = pytest.mark.gpu


def f2(x):
    return (x[0] - 0.3) ** 2 + (x[1] + 0.2) ** 2


def test_gp_phase_improves_and_respects_bounds():
    from mpi_opt_amd.optimizer import Optimizer

    opt = Optimizer([(-1.0, 1.0), (-1.0, 1.0)], n_initial_points=6, random_state=3,
                    acq_optimizer_kwargs={"n_points": 4000})
    for _ in range(14):
        x = opt.ask()
        assert -1 <= x[0] <= 1 and -1 <= x[1] <= 1
        opt.tell(x, f2(x))
    best_random = min(opt.yi[:6])
    assert min(opt.yi) < best_random
    assert len(opt.models) == 9
    assert hasattr(opt, "gains_") and opt.gains_.shape == (3,)


def test_sampling_proposal_is_the_oracle_argmin():
    """acq_optimizer='sampling', acq_func='EI': the proposal is the candidate with
    the lowest -EI under the fitted GP, checked against the oracle posterior."""
    from mpi_opt_amd.optimizer import Optimizer

    opt = Optimizer([(0.0, 1.0), (0.0, 1.0), (0.0, 1.0)], n_initial_points=8, random_state=5,
                    acq_func="EI", acq_optimizer="sampling", acq_optimizer_kwargs={"n_points": 3000})
    rng = np.random.RandomState(0)
    X = rng.uniform(size=(8, 3)).tolist()
    y = [float(np.sin(3 * a) + b * c) for a, b, c in X]
    # replay the rng stream the optimizer will use for its candidates
    opt.tell(X, y)
    m = opt.models[-1]
    st = O.gp_from_theta(np.asarray(X), np.asarray(y), m.amp, m.length_scale, m.noise)
    # candidates the optimizer sampled: regenerate from the same rng state is not
    # possible after the fact, so score the proposal against a dense random set
    C = O.synthetic_candidates(20000, 3, seed=9)
    mu, sd = O.posterior_skopt(st, C)
    ei_best = O.gaussian_ei(mu, sd, min(y)).max()
    mu_p, sd_p = O.posterior_skopt(st, np.asarray([opt._next_x]))
    ei_p = O.gaussian_ei(mu_p, sd_p, min(y))[0]
    assert ei_p > 0.5 * ei_best


def test_cl_min_batch_ask():
    from mpi_opt_amd.optimizer import Optimizer

    opt = Optimizer([(10, 50), (2, 10), (0.0, 1.0)], n_initial_points=5, random_state=7,
                    acq_optimizer_kwargs={"n_points": 2000})
    X = opt.ask(5)
    opt.tell(X, [float(x[0] / 50 + x[2]) for x in X])
    batch = opt.ask(3)
    assert len(batch) == 3 and len({tuple(b) for b in batch}) == 3


def test_pickle_roundtrip_after_fit(tmp_path):
    import pickle

    from mpi_opt_amd.optimizer import Optimizer

    opt = Optimizer([(0.0, 1.0), (0.0, 1.0)], n_initial_points=4, random_state=1,
                    acq_optimizer_kwargs={"n_points": 1000})
    for _ in range(6):
        x = opt.ask()
        opt.tell(x, f2(x))
    p = tmp_path / "o.pkl"
    p.write_bytes(pickle.dumps(opt))
    o2 = pickle.loads(p.read_bytes())
    assert o2.ask() == opt.ask()
    x = o2.ask()
    o2.tell(x, f2(x))      # refits on the device after unpickling
    assert len(o2.models) == len(opt.models) + 1
