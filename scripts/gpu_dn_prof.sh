#!/bin/bash
# DenseNet leg alone under rocprofv3 --kernel-trace --stats; per-family summary
cd /tmp && rm -rf /tmp/dnp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/dnp -o dn --output-format csv -- \
    python "$GRAFT_REPO_ROOT/bench.py" --workload densenet --no-cpu-baseline --no-pmc > /tmp/dnp.log 2>&1 || { tail -5 /tmp/dnp.log; exit 1; }
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out/dnprof" && cp $(find /tmp/dnp -name "*kernel_stats.csv") "$GRAFT_REPO_ROOT/gpurun_out/dnprof/"
python3 - <<'PY'
import csv, glob, re, os
f = glob.glob(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/dnprof/*kernel_stats.csv")[0]
rows = [r for r in csv.DictReader(open(f)) if "::dn_" in r["Name"]]
tot = sum(float(r["TotalDurationNs"]) for r in rows)
agg = {}
for r in rows:
    k = re.search(r"::(dn_\w+)", r["Name"]).group(1)
    agg[k] = agg.get(k, 0) + float(r["TotalDurationNs"])
print("total dn ms", round(tot / 1e6, 2))
for k, v in sorted(agg.items(), key=lambda x: -x[1]):
    print("%-26s %8.2f ms %5.1f%%" % (k, v / 1e6, 100 * v / tot))
PY
