#!/bin/bash
# round 3: FETCH_SIZE / WRITE_SIZE calibration per access width (scripts/probes/fetch_calib.hip)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ae}
P=$GRAFT_REPO_ROOT/scripts/probes/fetch_calib
timeout -k 10 60 $P > gpurun_out/fetch_calib_${T}.log 2>&1 && cat gpurun_out/fetch_calib_${T}.log && \
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/calib_fetch_${T} -o pmc --output-format csv -- $P > $GRAFT_REPO_ROOT/gpurun_out/calib_fetch_${T}.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/calib_write_${T} -o pmc --output-format csv -- $P > $GRAFT_REPO_ROOT/gpurun_out/calib_write_${T}.log 2>&1 && \
cd $GRAFT_REPO_ROOT && python3 - <<PY
import csv, glob
for c in ("fetch", "write"):
    p = glob.glob("gpurun_out/calib_%s_${T}/**/*counter_collection.csv" % c, recursive=True)[0]
    for r in csv.DictReader(open(p)):
        v = float(r["Counter_Value"]) * 1024
        print("%-6s %-40s %-11s %.4f GiB (x%.3f of 1 GiB)" % (c, r["Kernel_Name"][:40], r["Counter_Name"], v / 2**30, v / 2**30))
PY
