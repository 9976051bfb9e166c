"""Run the option3 search (mpi_opt_amd.search) once and write its report as JSON,
with a progress line per trained epoch and per population (long runs on the GPU
box print at least once a minute).

    python scripts/search_run.py OUT.json [search CLI flags ...]
"""
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import scripts.ab_lib  # noqa: E402,F401 -- MPO_LIB_AB: another build's libmpo.so (same-box A/B)


def main():
    out_path, argv = sys.argv[1], sys.argv[2:]
    import random

    from mpi_opt_amd import search

    random.seed(0)
    args = search.make_parser().parse_args(argv)
    t0 = time.perf_counter()

    def log(*m):
        print(f"[{time.perf_counter() - t0:7.1f} s]", *m, file=sys.stderr, flush=True)

    partial = {"argv": argv, "populations": []}

    def population_done(i, entry, stats):
        # a partial report after every population (a run cut short still leaves its timeline)
        partial["populations"].append({"index": i, "trials": entry[3], "before_s": entry[0], "wait_s": entry[1],
                                       "train_s": entry[2], "t_s": time.perf_counter() - t0,
                                       "refits": stats["refits"], "refit_n_sum": stats["n_sum"],
                                       "refit_s": stats["refit_s"], "propose_s": stats["propose_s"]})
        with open(out_path + ".partial", "w") as fh:
            json.dump(partial, fh, indent=1, default=float)

    import threading

    from mpi_opt_amd import optimizer as O

    stop = threading.Event()

    def heartbeat():   # a line a minute, whatever phase the search is in
        while not stop.wait(60.0):
            log(f"heartbeat: {O.STATS['refits']} refits so far")

    threading.Thread(target=heartbeat, daemon=True).start()
    with tempfile.TemporaryDirectory() as tmp:
        if args.checkpoint == "coordinator.pkl":
            args.checkpoint = os.path.join(tmp, "coordinator.pkl")
        rep = search.run_search(args, log=log, progress=log, on_population=population_done)
    stop.set()
    if rep is None:
        return 0
    rep["argv"] = argv
    gp = rep["gp"]
    samples = gp.pop("samples")
    gp["refit_n_hist"] = {str(k): int(v) for k, v in zip(*__import__("numpy").unique(
        [n for n, _ in samples], return_counts=True))} if samples else {}
    rep["gp_refit_mean_n"] = gp["n_sum"] / max(1, gp["refits"])
    rep["refits_per_optimizer_s"] = gp["refits"] / max(1e-9, rep["optimizer_s"])
    with open(out_path, "w") as fh:
        json.dump(rep, fh, indent=1, default=float)
    keys = ("wall_s", "trials_told", "trials_trained", "populations", "trials_per_hour", "trained_per_hour",
            "optimizer_s", "ask_s", "tell_s", "chain_wait_s", "chain_busy_s", "train_s", "gp_refit_mean_n",
            "refits_per_optimizer_s")
    print(json.dumps({k: rep[k] for k in keys} | {"refits": gp["refits"]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
