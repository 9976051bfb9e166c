#!/bin/bash
# r06 session u: a lone chain's round turnaround (device idle between LML rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/u_tr -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/scripts/ask_chain_probe.py" --ask-n 16 --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/u_chain.log" 2>&1 ) && \
python3 scripts/chain_gaps.py "$(find /tmp/u_tr -name '*kernel_trace.csv' | head -1)" > gpurun_out/u_gaps.log 2>&1
