"""Read a rocprofv3 kernel_trace.csv of scripts/lml_round_prof.py: per LML round
(a run of consecutive dispatches starting at the round's first kernel), the
summed kernel durations, the span from the first start to the last end, and
the mean duration of each kernel.  Usage: lml_round_gaps.py TRACE.csv FIRST_KERNEL"""
import collections
import csv
import re
import sys


def main():
    path, first = sys.argv[1], sys.argv[2]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rounds, cur = [], []
    for r in rows:
        name = r["Kernel_Name"]
        if first in name and cur:
            rounds.append(cur)
            cur = []
        if first in name or cur:
            cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if cur:
        rounds.append(cur)
    rounds = rounds[20:]       # past the warm-up
    if not rounds:
        print("no rounds")
        return
    busy = [sum(e - s for _, s, e in rd) for rd in rounds]
    span = [rd[-1][2] - rd[0][1] for rd in rounds]
    gaps = [rounds[i + 1][0][1] - rounds[i][-1][2] for i in range(len(rounds) - 1)]
    per = collections.defaultdict(list)
    for rd in rounds:
        for name, s, e in rd:
            m = re.search(r"::(\w+)", name)
            per[m.group(1) if m else name[:48]].append(e - s)
    print(f"{len(rounds)} rounds, {len(rounds[0])} kernels each: kernel time {sum(busy) / len(busy) / 1e3:.1f} us, "
          f"span {sum(span) / len(span) / 1e3:.1f} us, between rounds {sum(gaps) / max(1, len(gaps)) / 1e3:.1f} us")
    for k, v in per.items():
        print(f"  {k:50s} {sum(v) / len(v) / 1e3:7.2f} us x {len(v) / len(rounds):.0f}")


if __name__ == "__main__":
    main()
