"""The CLI keeps option3's flags and defaults (hyperparameter_search_option3.py:54-96),
pinned by tests/golden/reference_cli_mnist.json: the reference's own
``make_parser()`` run in the build container under recording stand-ins for its
imports (tests/golden/make_reference_cli_mnist_fixture.py)."""
import argparse
import json
import os

import pytest

from mpi_opt_amd.search import block_layout, check_sanity, check_training_flags, main, make_parser
from tests.conftest import GOLDEN

FIXTURE = json.load(open(os.path.join(GOLDEN, "reference_cli_mnist.json")))


def test_defaults_match_reference():
    a = vars(make_parser().parse_args([]))
    for k, v in FIXTURE["defaults"].items():
        assert a[k] == v, k


def test_every_reference_flag_is_kept():
    """Option strings, dest, default, type and action of every flag the
    reference's parser defines; this build's flags are additions."""
    ours = {tuple(a.option_strings): a for a in make_parser()._actions if not isinstance(a, argparse._HelpAction)}
    for ref in FIXTURE["parser"]:
        a = ours.get(tuple(ref["option_strings"]))
        assert a is not None, ref["option_strings"]
        assert a.dest == ref["dest"] and a.default == ref["default"], ref["option_strings"]
        assert getattr(a.type, "__name__", None) == ref["type"] and type(a).__name__ == ref["action"]
        assert (list(a.choices) if a.choices else None) == ref["choices"], ref["option_strings"]


def test_training_flags_are_honoured_or_refused():
    """--loss / --optimizer / --early-stopping / --target-metric reach the trainer
    (option3:60-61, 66-69) or stop the CLI with status 2 -- never silently ignored."""
    p = make_parser()
    assert check_training_flags(p.parse_args([])) is None
    rule = check_training_flags(p.parse_args(["--loss", "categorical_crossentropy", "--optimizer", "sgd",
                                              "--early-stopping", "3", "--target-metric", "val_acc,>,0.97"]))
    assert rule.patience == 3 and rule.target == ("val_acc", ">", 0.97)
    for bad in (["--loss", "mse"], ["--optimizer", "rmsprop"], ["--early-stopping", "soon"],
                ["--target-metric", "val_acc>0.9"]):
        with pytest.raises(ValueError):
            check_training_flags(p.parse_args(bad))
        assert main(bad) == 2


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


def test_no_effect_flags_are_reported_not_silent():
    """mpi_learn's asynchronous-exchange flags have no counterpart here: set away
    from their defaults they produce a note (and their --help says so)."""
    from mpi_opt_amd import search

    p = search.make_parser()
    assert search.no_effect_notes(p.parse_args([])) == []
    notes = search.no_effect_notes(p.parse_args(["--easgd", "--sync-every", "4", "--elastic-lr", "0.5"]))
    assert len(notes) == 3 and all("no effect" in n for n in notes)
    helps = {a.dest: a.help or "" for a in p._actions}
    for dest, _ in search.NO_EFFECT_FLAGS:
        assert "no effect" in helps[dest], dest
