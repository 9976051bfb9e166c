"""Run bench.py's configs[0] search twice in one process and compare the runs
(diagnostic, ``--seed S`` seeds the block shuffle: are the trained trials, their fold losses and the training time
reproducible from run to run?)."""
import json
import os
import random
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_opt_amd import search  # noqa: E402

ARGV = ["--world-size", "21", "--block-size", "5", "--epochs", "10", "--num-iterations", "10",
        "--n-fold", "5", "--n-samples", "60000", "--synthetic-labels", "learnable"]


def one(extra, seed):
    if seed is not None:
        random.seed(seed)       # the scheduler's block shuffle (bench.py seeds it)
    a = search.make_parser().parse_args(ARGV + extra)
    with tempfile.TemporaryDirectory() as tmp:
        a.checkpoint = os.path.join(tmp, "coordinator.pkl")
        t0 = time.perf_counter()
        rep = search.run_search(a, log=lambda *_: None)
        rep["outer_s"] = time.perf_counter() - t0
    return rep


def main():
    extra = sys.argv[1:]
    seed = None
    if extra[:1] == ["--seed"]:
        seed, extra = int(extra[1]), extra[2:]
    reps = [one(extra, seed) for _ in range(2)]
    for r in reps:
        print(json.dumps({"wall_s": r["wall_s"], "train_s": r["train_s"], "populations": r["populations"],
                          "best_fom": r["best_fom"], "told_foms": r["told_foms"]}), flush=True)
    same_params = reps[0]["trained_params"] == reps[1]["trained_params"]
    same_foms = reps[0]["told_foms"] == reps[1]["told_foms"]
    print("same trained params:", same_params, " same told foms:", same_foms)
    if not same_params:
        for p, q in zip(reps[0]["trained_params"], reps[1]["trained_params"]):
            print(p, q)


if __name__ == "__main__":
    main()
