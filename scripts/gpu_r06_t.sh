#!/bin/bash
# r06 session t: where the configs[0] search leg's 46 s go (kernel stats of the whole leg)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/t_pr -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --workload search --no-cpu-baseline --no-pmc \
    > "$GRAFT_REPO_ROOT/gpurun_out/t_search.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/t_search.err" ) && \
cp "$(find /tmp/t_pr -name '*kernel_stats.csv' | head -1)" gpurun_out/t_kernel_stats.csv
