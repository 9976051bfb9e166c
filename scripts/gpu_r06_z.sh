#!/bin/bash
# r06 session z: launch cost of a 3.3 KB by-value kernel argument
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/probes/launch_lat > gpurun_out/z2_launch.log 2>&1 && \
true
