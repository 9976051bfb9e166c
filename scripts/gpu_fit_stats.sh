#!/bin/bash
# per-kernel rocprof stats of the split-sweep LML at one n (default 500)
cd /tmp
rm -rf /tmp/fs
MPO_FIT_KERNEL=split timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/fs -o fit --output-format csv -- \
    python "$GRAFT_REPO_ROOT/scripts/fit_probe.py" --n ${N:-500} --kernels split --reps 0 > /tmp/fs.log 2>&1 || { tail -5 /tmp/fs.log; exit 1; }
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out/fitstats" && cp $(find /tmp/fs -name "*kernel_stats.csv") "$GRAFT_REPO_ROOT/gpurun_out/fitstats/"
cut -d, -f1-4 $(find /tmp/fs -name "*kernel_stats.csv")
