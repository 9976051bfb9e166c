#!/bin/bash
# r06 session s: host vs device time of a small population's train step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/host_step_probe.py --trials 2 4 8 64 > gpurun_out/s_host.log 2>&1 && \
MPO_POP_PLAN=streams=1 timeout -k 10 300 python -u scripts/host_step_probe.py --trials 2 4 > gpurun_out/s_host_s1.log 2>&1
