#!/bin/bash
# DenseNet probe under rocprofv3 kernel stats (serial: one stream), r05.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dn}
( cd /tmp && rm -rf /tmp/prof_$TAG && MPO_DN_PLAN=${PLAN:-streams=1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG \
    -o run --output-format csv -- python "$GRAFT_REPO_ROOT/scripts/dn_probe.py" --steps 10 \
    > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 ) && \
mkdir -p gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$TAG/ \; && \
echo "PROF OK" && tail -2 gpurun_out/prof_$TAG.log
