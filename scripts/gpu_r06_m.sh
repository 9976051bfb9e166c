#!/bin/bash
# r06 session m: pivot-sweep latency micro-probe; one LML round's kernel trace at n = 288
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/probes/sweep_lat > gpurun_out/m_sweep_lat.log 2>&1 && \
( cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -d /tmp/m_tr -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/scripts/lml_round_prof.py" 288 > "$GRAFT_REPO_ROOT/gpurun_out/m_round.log" 2>&1 ) && \
python3 scripts/lml_round_gaps.py "$(ls /tmp/m_tr/*/*kernel_trace.csv | head -1)" sw_xs_build > gpurun_out/m_gaps.log 2>&1
