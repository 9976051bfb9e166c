"""Split a lone chain's round turnaround (rocprofv3 --kernel-trace --hip-runtime-trace
of scripts/ask_chain_probe.py) into: the last kernel's end -> hipStreamSynchronize
returns; that return -> the next round's first hipLaunchKernel call; that call's
entry -> its kernel's start on the device.

    python scripts/chain_api_gaps.py KERNEL_TRACE.csv HIP_API_TRACE.csv
"""
import bisect
import csv
import sys

import numpy as np


def main():
    kt = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    api = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt]
    syncs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api if r["Function"] == "hipStreamSynchronize"]
    launches = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in api
                if r["Function"] in ("hipLaunchKernel", "hipExtLaunchKernel", "hipModuleLaunchKernel")]
    sync_end = sorted(e for _, e in syncs)
    launch_start = sorted(s for s, _ in launches)
    a, b, c, tot, lcall = [], [], [], [], []
    for i in range(1, len(ev)):
        if "sw_xs_build" not in ev[i][0] or "sw_pairs_final" not in ev[i - 1][0]:
            continue
        k_end, k_next = ev[i - 1][2], ev[i][1]
        j = bisect.bisect_left(sync_end, k_end)          # the sync that returned after the last kernel ended
        if j >= len(sync_end) or sync_end[j] > k_next:
            continue
        se = sync_end[j]
        m = bisect.bisect_left(launch_start, se)         # the next launch call after it
        if m >= len(launch_start) or launch_start[m] > k_next:
            continue
        ls = launch_start[m]
        a.append(se - k_end)
        b.append(ls - se)
        c.append(k_next - ls)
        tot.append(k_next - k_end)
        lcall.append(launches[[s for s, _ in launches].index(ls)][1] - ls)
    f = lambda v: f"{np.median(v) / 1e3:.1f}"   # noqa: E731
    print(f"{len(tot)} turnarounds, median us: total {f(tot)} = kernel end -> sync returns {f(a)} + host (L-BFGS-B, "
          f"batcher, next launch setup) {f(b)} + launch call -> kernel start {f(c)}; the launch call itself {f(lcall)}")


if __name__ == "__main__":
    main()
