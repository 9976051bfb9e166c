"""Per-kernel-family totals of every counter in a rocprofv3 --pmc csv (diagnostic)."""
import collections
import csv
import glob
import sys

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from pmc_summary import family  # noqa: E402

path = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(path)):
    key = family(r["Kernel_Name"])
    if key is None:
        continue
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[key].add(r.get("Dispatch_Id", ""))
for key, d in sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
    n = max(1, len(disp[key]))
    print("%-18s launches=%d " % (key, n) + " ".join("%s=%.4g" % (c, v / n) for c, v in sorted(d.items())))
