#!/bin/bash
# r06 session n: an LML sweep step's timestamps; one round's kernel trace at n = 288 / 448
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MPO_FIT_DEBUG=24 timeout -k 10 120 python -u scripts/step_stamps_probe.py 96 288 448 > gpurun_out/n_stamps.log 2>&1 && \
( cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -d /tmp/n_tr -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/scripts/lml_round_prof.py" 288 > "$GRAFT_REPO_ROOT/gpurun_out/n_round.log" 2>&1 ) && \
find /tmp/n_tr -name "*kernel_trace.csv" > gpurun_out/n_files.log && \
python3 scripts/lml_round_gaps.py "$(find /tmp/n_tr -name '*kernel_trace.csv' | head -1)" sw_xs_build > gpurun_out/n_gaps.log 2>&1
