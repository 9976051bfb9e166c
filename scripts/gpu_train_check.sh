#!/bin/bash
# training parity tests, then the throughput probe + rocprof kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 && echo "TESTS OK" && bash scripts/gpu_train_prof.sh
