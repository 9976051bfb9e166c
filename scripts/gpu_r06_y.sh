#!/bin/bash
# r06 session y: a lone chain's round turnaround split with the HIP runtime trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace -d /tmp/y_tr -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/scripts/ask_chain_probe.py" --ask-n 16 --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/y_chain.log" 2>&1 ) && \
find /tmp/y_tr -name "*.csv" > gpurun_out/y_files.log && \
python3 scripts/chain_api_gaps.py "$(find /tmp/y_tr -name '*kernel_trace.csv' | head -1)" "$(find /tmp/y_tr -name '*hip_api_trace.csv' | head -1)" > gpurun_out/y_gaps.log 2>&1
