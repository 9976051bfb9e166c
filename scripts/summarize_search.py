"""Summarise search_run.py reports (JSON) side by side: wall, told / trained trials
per hour, the optimizer vs training split, refits and their rate, and the
per-population timeline.

    python scripts/summarize_search.py gpurun_out/s3_w0_b.json gpurun_out/s3_w4_b.json ...
"""
import json
import sys


def main():
    rows = []
    for fn in sys.argv[1:]:
        r = json.load(open(fn))
        rows.append((fn, r))
        print(f"== {fn}: {' '.join(r.get('argv', []))}")
        print(f"   wall {r['wall_s']:.1f} s   told {r['trials_told']} ({r['trials_per_hour']:.0f}/h)   "
              f"trained {r['trials_trained']} ({r['trained_per_hour']:.0f}/h)   populations {r['populations']}")
        print(f"   optimizer {r['optimizer_s']:.1f} s (ask {r['ask_s']:.1f}, tell {r['tell_s']:.1f}, "
              f"chain wait {r.get('chain_wait_s', 0):.1f}; chain busy {r.get('chain_busy_s', 0):.1f} worker-s, "
              f"{r.get('chain_workers')} {r.get('chain_pool')})   training {r['train_s']:.1f} s")
        gp = r["gp"]
        print(f"   refits {gp['refits']} (mean n {r.get('gp_refit_mean_n', 0):.0f}, max {gp['n_max']}), "
              f"{r.get('refits_per_optimizer_s', 0):.1f} per optimizer-second; per refit (worker-thread ms): "
              f"fit {1e3 * gp['refit_s'] / max(1, gp['refits']):.1f}, proposal {1e3 * gp['propose_s'] / max(1, gp['refits']):.1f}")
        for k, t in enumerate(r.get("timeline", [])):
            print(f"   population {k}: {t[3]} trials; before it {t[0]:.1f} s, waiting for ask batches {t[1]:.1f} s, "
                  f"training {t[2]:.1f} s")


if __name__ == "__main__":
    main()
