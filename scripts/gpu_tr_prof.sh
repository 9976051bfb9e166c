#!/bin/bash
# Training leg alone under rocprofv3 --kernel-trace --stats (VAR=name, extra env via ENVS)
set -o pipefail
V=${VAR:-a}
cd /tmp && rm -rf /tmp/trp_$V && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/trp_$V -o tr --output-format csv -- \
    python "$GRAFT_REPO_ROOT/bench.py" --workload train --no-cpu-baseline --no-pmc > /tmp/trp_$V.log 2>&1 || { tail -5 /tmp/trp_$V.log; exit 1; }
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out/trprof" && cp $(find /tmp/trp_$V -name "*kernel_stats.csv") "$GRAFT_REPO_ROOT/gpurun_out/trprof/tr_$V.csv"
