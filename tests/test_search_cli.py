"""The CLI keeps option3's flags and defaults (hyperparameter_search_option3.py:54-96)."""
from mpi_opt_amd.search import block_layout, check_sanity, main, make_parser

REFERENCE_DEFAULTS = dict(verbose=False, batch=100, epochs=10, optimizer="adam", loss="binary_crossentropy",
                          sync_every=1, data_preload=0, caching_dir="", early_stopping=None, target_metric=None,
                          easgd=False, worker_optimizer="sgd", elastic_force=0.9, elastic_lr=1.0,
                          elastic_momentum=0, block_size=2, n_fold=1, n_master=1, n_process=1, num_iterations=10,
                          previous_state=None, target_objective=None, example="mnist")


def test_defaults_match_reference():
    a = make_parser().parse_args([])
    for k, v in REFERENCE_DEFAULTS.items():
        assert getattr(a, k) == v, k


def test_readme_invocation_parses():
    a = make_parser().parse_args("--block-size 5 --example mnist --epochs 10 --num-iterations 10 --n-fold 5".split())
    assert (a.block_size, a.epochs, a.num_iterations, a.n_fold) == (5, 10, 10, 5)


def test_block_arithmetic():
    assert block_layout(21, 5) == (4, 0)      # README: 1 opt master + 4 blocks x 5
    assert block_layout(101, 5) == (20, 0)
    assert block_layout(20, 5) == (3, 4)


def test_sanity_and_leftover_exit():
    import pytest

    with pytest.raises(AssertionError):
        check_sanity(make_parser().parse_args(["--block-size", "1"]))
    assert main(["--block-size", "5", "--world-size", "20"]) == 1
    assert main(["--example", "gan"]) == 2
