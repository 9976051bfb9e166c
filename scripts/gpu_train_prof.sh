#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/train_probe.py ${ARGS} > gpurun_out/train_probe.log 2>&1 && cat gpurun_out/train_probe.log && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/tprof" -o train \
    --output-format csv -- python "$GRAFT_REPO_ROOT/scripts/train_probe.py" --steps 3 ${ARGS} \
    > "$GRAFT_REPO_ROOT/gpurun_out/tprof.log" 2>&1 ) && echo "PROF OK"
