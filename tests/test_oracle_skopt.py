"""CPU checks of the skopt ask/tell oracle (``oracle/skopt_optimizer.py``) and of
the host-side pieces the device Optimizer shares with it: the RandomState
stream of the random phase, the ``copy()`` hand-off of cl_min batches and the
candidate draws (``Space.rvs_transformed``)."""
import numpy as np

from oracle.skopt_optimizer import SkoptOracle


def _space():
    from mpi_opt_amd.models import mnist_space

    return mnist_space()


def test_candidate_draws_match_the_oracle_space():
    from mpi_opt_amd.space import Space

    ora = SkoptOracle(_space(), random_state=0)
    a = Space(_space()).rvs_transformed(n_samples=4000, random_state=np.random.RandomState(11))
    b = ora.space.transform(ora.space.rvs(4000, np.random.RandomState(11)))
    np.testing.assert_array_equal(a, b)


def test_random_phase_and_copy_handoff_match_product_optimizer():
    """Before the GP is reached both sides only consume the RandomState: the
    constructor's estimator seed, the random points, and ``ask(n)``'s
    ``copy(random_state=rng.randint(...))`` -- sequences must be identical."""
    from mpi_opt_amd.optimizer import Optimizer

    opt = Optimizer(_space(), random_state=13579, n_initial_points=100, base_estimator="dummy")
    ora = SkoptOracle(_space(), random_state=13579, n_initial_points=100)
    assert opt._gp_seed == ora.gp_seed
    for i in range(6):
        a, b = opt.ask(), ora.ask()
        assert a == b, (i, a, b)
        opt.tell(a, float(i))
        ora.tell(b, float(i))
    assert opt.ask(4) == ora.ask(4)
    assert opt.ask() == ora.ask()


def test_oracle_loop_reaches_the_gp_and_caches_batches():
    ora = SkoptOracle(_space(), random_state=3, n_initial_points=4, n_points=400)
    for i in range(6):
        x = ora.ask()
        ora.tell(x, float((x[0] - 30) ** 2 / 100 + x[4]))
    assert len(ora.trace) == 3 and len(ora.models) == 3
    rec = ora.trace[-1]
    assert set(rec["top"]) == {"EI", "LCB", "PI"} and all(len(v) == 5 for v in rec["top"].values())
    assert np.all(rec["gains"] != 0.0)            # gp_hedge gains updated after the first proposal
    batch = ora.ask(3)
    assert ora.ask(3) is batch                    # cached until the next tell
    assert len(ora.batch_trace) == 1 + 3          # copy() refit + one refit per lie
    assert len({tuple(b) for b in batch}) == 3
    ora.tell(batch[0], 0.5)
    assert ora.cache_ == {}
