"""Read a rocprofv3 kernel_trace.csv of scripts/ask_chain_probe.py: per LML round
of the lone chain (sw_xs_build_kernel .. sw_pairs_final_kernel), the kernel time,
the span, and the device-idle gap from one round's last kernel to the next
round's first (the host turnaround: completion seen, L-BFGS-B step, next launch).
Rounds separated by other kernels (the proposal's scoring / polish) are skipped.

    python scripts/chain_gaps.py TRACE.csv
"""
import csv
import sys

import numpy as np


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    rounds, cur = [], None
    for name, s, e in ev:
        if "sw_xs_build" in name:
            cur = [(name, s, e)]
        elif cur is not None:
            cur.append((name, s, e))
            if "sw_pairs_final" in name:
                rounds.append(cur)
                cur = None
    gaps = []
    for a, b in zip(rounds, rounds[1:]):
        g = b[0][1] - a[-1][2]
        # consecutive rounds of one fit: nothing else ran between them
        between = [x for x in ev if a[-1][2] <= x[1] < b[0][1]]
        if not between:
            gaps.append(g)
    busy = [sum(e - s for _, s, e in rd) for rd in rounds]
    span = [rd[-1][2] - rd[0][1] for rd in rounds]
    print(f"{len(rounds)} rounds: kernel time median {np.median(busy) / 1e3:.1f} us, span {np.median(span) / 1e3:.1f} us; "
          f"turnaround (device idle between consecutive rounds) median {np.median(gaps) / 1e3:.1f} us, "
          f"p10 {np.percentile(gaps, 10) / 1e3:.1f}, p90 {np.percentile(gaps, 90) / 1e3:.1f} ({len(gaps)} gaps)")


if __name__ == "__main__":
    main()
