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
    assert len(files) >= 2 * 9                      # one per (trial, fold)
    doc = json.loads(files[0].read_text())
    assert list(doc["history"]) == ["0"] and len(doc["history"]["0"]["val_loss"]) == 1
    assert doc["meta"]["fold"] in (0, 1)


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
    files = sorted((tmp_path / "hist").iterdir())
    assert len(files) == 10 * 5                     # one per (trial, fold): meta.fold = manager.fold_num
    docs = [json.loads(f.read_text()) for f in files]
    assert sorted(d["meta"]["fold"] for d in docs) == sorted(list(range(5)) * 10)
    doc = docs[0]
    assert list(doc["history"]) == ["0"] and len(doc["history"]["0"]["val_loss"]) == 2
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
    assert doc["meta"]["fold"] == 0
    # 77 train samples (a + b) -> 7 steps of 10, 50 validation samples (c) -> 5 batches
    assert h["dropped_train_samples"] == 7 and h["dropped_val_samples"] == 0


def _search3(tmp_path, workers):
    from mpi_opt_amd import optimizer as O
    from mpi_opt_amd import search

    random.seed(3)
    args = search.make_parser().parse_args(
        ["--world-size", "17", "--block-size", "2", "--n-fold", "5", "--num-iterations", "32", "--epochs", "1",
         "--n-samples", "2500", "--chain-workers", str(workers),
         "--checkpoint", str(tmp_path / f"c{workers}.pkl")])
    rep = search.run_search(args)
    rep["refit_ns"] = sorted(n for n, _ in O.STATS["samples"])
    return rep


def test_configs3_layout_concurrent_chains_equal_sequential(tmp_path):
    """BASELINE configs[3]'s layout (-n 2k+1 --block-size 2 --n-fold 5, a fresh
    cl_min ask(num_iterations) after every tell, coordinator.py:46-50, 73) at
    reduced size: 8 blocks, 32 iterations, 1 epoch on 2 500 samples.  The ask
    batches run on 4 concurrent chains (mpi_opt_amd.chains) and inline: the told
    points, their FOMs, every trained trial and the populations are identical,
    and the GP refits are exactly the protocol's (bench.protocol_refits replays
    it with a refit-counting optimizer: count and observation numbers)."""
    import bench

    seq = _search3(tmp_path, 0)
    par = _search3(tmp_path, 4)
    want_refits, want_pops = bench.protocol_refits(17, 2, 32)
    for rep in (seq, par):
        assert rep["populations"] == want_pops == [8, 8, 8, 8]
        assert rep["trials_told"] == 24 and rep["trials_trained"] == 32 and rep["tail_trials"] == 8
        assert rep["gp"]["refits"] == len(want_refits)
        assert rep["refit_ns"] == sorted(want_refits)
    assert par["told_params"] == seq["told_params"] and par["told_foms"] == seq["told_foms"]
    assert par["trained_params"] == seq["trained_params"]
    assert par["best_fom"] == seq["best_fom"] and par["best_params"] == seq["best_params"]
    assert par["chain_wait_s"] > 0 and seq["chain_wait_s"] == 0


def _nccl_search3_worker(port, tmp, q):
    """One rank over RCCL: the configs[3] layout through DistributedEvaluator,
    DistributedChainExecutor and ShardedScorer, plus one sharded scoring round."""
    import pathlib
    import types

    import numpy as np
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        rep = _search3(pathlib.Path(tmp), 4)
        from mpi_opt_amd.blocks import DistributedEvaluator, local_topk

        rng = np.random.RandomState(4)
        req = {"Xt": rng.rand(40, 5), "y": rng.rand(40), "amp": 1.3, "ls": np.full(5, 0.4), "noise": 1e-5,
               "cand": rng.rand(20000, 5), "y_opt": 0.01, "acqs": ["EI", "LCB", "PI"], "xi": 0.01,
               "kappa": 1.96, "k": 5}
        ev = DistributedEvaluator(types.SimpleNamespace(device=torch.device("cuda", 0)))
        got = ev.score(req)            # broadcast + all_gather of the top-k over RCCL
        want = local_topk(req, 0, len(req["cand"]), device=torch.device("cuda", 0))
        score_ok = all(np.array_equal(got[a][1], want[a][1]) and np.array_equal(got[a][0], want[a][0])
                       for a in req["acqs"])
        # a fitted model's round: its prepared factor crosses RCCL as raw words
        from mpi_opt_amd.optimizer import GPModel

        est = GPModel(req["Xt"], req["y"], req["amp"], req["ls"], req["noise"], device=torch.device("cuda", 0))
        fac = ev.score({"est": est, **{k: req[k] for k in ("cand", "y_opt", "acqs", "xi", "kappa", "k")}})
        score_ok = score_ok and all(np.array_equal(fac[a][1], want[a][1]) and np.array_equal(fac[a][0], want[a][0])
                                    for a in req["acqs"])
        maps = open("/proc/self/maps").read()
        rccl = sorted({ln.split()[-1] for ln in maps.splitlines() if "librccl" in ln})
        q.put({k: rep[k] for k in ("told_params", "told_foms", "trained_params", "populations", "best_fom",
                                   "best_params", "refit_ns")}
              | {"refits": rep["gp"]["refits"], "backend": dist.get_backend(), "rccl": rccl,
                 "score_ok": bool(score_ok)})
    finally:
        dist.destroy_process_group()


def test_configs3_layout_over_rccl_equals_one_process(tmp_path):
    """the configs[3] path's collectives on RCCL.  A world-size-1
    ``nccl`` group (the 1-GPU box cannot host two RCCL ranks) runs the search with
    the distributed evaluator, the chains dealt over the ranks and the sharded
    scorer: every broadcast_object_list / all_gather_object goes through RCCL's
    device-tensor staging (the reference's send / irecv exchange,
    coordinator.py:140-150, option3:172-205).  Told points, FOMs, trained trials
    and the refit multiset equal the non-distributed run; a sharded scoring round
    returns the single-device top-k bit for bit."""
    import torch.multiprocessing as mp

    s = __import__("socket").socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_search3_worker, args=(port, str(tmp_path), q))
    p.start()
    got = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert got["backend"] == "nccl" and got["rccl"], "RCCL was not loaded"
    assert got["score_ok"]
    want = _search3(tmp_path, 4)
    assert got["populations"] == want["populations"] == [8, 8, 8, 8]
    assert got["told_params"] == want["told_params"] and got["told_foms"] == want["told_foms"]
    assert got["trained_params"] == want["trained_params"]
    assert got["refits"] == want["gp"]["refits"] and got["refit_ns"] == want["refit_ns"]
    assert got["best_fom"] == want["best_fom"] and got["best_params"] == want["best_params"]
