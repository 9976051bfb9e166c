"""The whole option3 loop on the GPU: Coordinator + PopulationComm + device trials."""
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu


def test_search_cli_end_to_end(tmp_path, monkeypatch):
    from mpi_opt_amd import search

    monkeypatch.chdir(tmp_path)
    random.seed(0)
    rc = search.main(["--block-size", "2", "--world-size", "7", "--epochs", "1", "--num-iterations", "12",
                      "--n-samples", "1000", "--n-fold", "2", "--history-dir", str(tmp_path / "hist")])
    assert rc == 0
    assert (tmp_path / "coordinator.pkl").exists()
    files = list((tmp_path / "hist").iterdir())
    assert len(files) >= 9
    doc = json.loads(files[0].read_text())
    assert len(doc["history"]) == 2 and len(doc["history"]["0"]["val_loss"]) == 1


def test_evaluator_is_deterministic():
    from mpi_opt_amd.blocks import TrialEvaluator
    from mpi_opt_amd.models import BuilderFromFunction, mnist_space
    from mpi_opt_amd.models import test_mnist as mnist_fn
    from mpi_opt_amd.population import synthetic_mnist

    x, y = synthetic_mnist(1000, seed=1)
    params = [[10, 2, 2, 50, 0.1], [25, 4, 3, 80, 0.7], [50, 10, 10, 200, 0.2]]
    a = TrialEvaluator(BuilderFromFunction(mnist_fn, mnist_space()), x, y, n_fold=2, epochs=1).evaluate(params)
    # a different batching of the same trials gives identical FOMs
    ev = TrialEvaluator(BuilderFromFunction(mnist_fn, mnist_space()), x, y, n_fold=2, epochs=1)
    units = ev.units(params)
    res = {}
    for u in units:
        res.update(ev.train_units([u]))
    b = ev.foms(params, res)
    assert a == b
    assert all(0.0 < f < 1.0 for f in a)


def test_configs0_search_shape(tmp_path, monkeypatch):
    """BASELINE configs[0]'s layout -- `-n 21 --block-size 5 --n-fold 5
    --num-iterations 10` -- end to end on reduced data (3000 samples, 2 epochs;
    the full 60k x 10-epoch run is bench.py's `search` leg).  4 blocks train as
    populations of 4, 4 and the 2-trial tail; 6 results are told (the reference
    leaves the last num_blocks trials untold); every trained trial writes its
    history JSON."""
    from mpi_opt_amd import search

    monkeypatch.chdir(tmp_path)
    random.seed(0)
    args = search.make_parser().parse_args(
        ["--world-size", "21", "--block-size", "5", "--epochs", "2", "--num-iterations", "10", "--n-fold", "5",
         "--n-samples", "3000", "--history-dir", str(tmp_path / "hist")])
    rep = search.run_search(args)
    assert rep["num_blocks"] == 4
    assert rep["populations"] == [4, 4, 2]
    assert rep["trials_trained"] == 10 and rep["trials_told"] == 6
    assert rep["train_s"] > 0 and rep["optimizer_s"] >= 0
    files = list((tmp_path / "hist").iterdir())
    assert len(files) == 10
    doc = json.loads(files[0].read_text())
    assert len(doc["history"]) == 5 and len(doc["history"]["0"]["val_loss"]) == 2
    assert doc["history"]["0"]["dropped_train_samples"] == 0


def test_search_reads_hdf5_data_dir(tmp_path, monkeypatch):
    """--data-dir: option3's mnist data layout (*.h5 with features / labels, 70 %
    of the files train, the rest validate), read by mpi_opt_amd.h5."""
    import shutil

    from mpi_opt_amd import search
    from tests.conftest import GOLDEN

    data = tmp_path / "mnist"
    data.mkdir()
    for fn in ("mnist_a.h5", "mnist_b.h5", "mnist_c.h5"):
        shutil.copy(os.path.join(GOLDEN, "h5", fn), data / fn)
    monkeypatch.chdir(tmp_path)
    random.seed(0)
    args = search.make_parser().parse_args(
        ["--world-size", "5", "--block-size", "2", "--epochs", "1", "--num-iterations", "3", "--batch", "10",
         "--data-dir", str(data), "--history-dir", str(tmp_path / "hist")])
    rep = search.run_search(args)
    assert rep["trials_trained"] == 3
    doc = json.loads(next((tmp_path / "hist").iterdir()).read_text())
    h = doc["history"]["0"]
    # 77 train samples (a + b) -> 7 steps of 10, 50 validation samples (c) -> 5 batches
    assert h["dropped_train_samples"] == 7 and h["dropped_val_samples"] == 0
