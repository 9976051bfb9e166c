"""Short per-kernel summary of a rocprofv3 *_kernel_stats.csv (diagnostic)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 16]:
    m = re.search(r"::(\w+(<[^>]*>)?)\(", r["Name"])
    print("%-36s %5s calls %8.3f ms/call %8.2f ms/step" % ((m.group(1) if m else r["Name"][:36]), r["Calls"],
          float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6 / div))
print("total %.2f ms/step" % (tot / 1e6 / div))
