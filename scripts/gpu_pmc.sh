#!/bin/bash
# One PMC pass over the train probe (counters in $PMC), csv under gpurun_out/pmc_$TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PROG=${PROG:-scripts/train_probe.py --steps 1}
( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc ${PMC} -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}" -o pmc \
    --output-format csv -- python $GRAFT_REPO_ROOT/$PROG > "$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}.log" 2>&1 ) && echo "PMC ${TAG} OK"
