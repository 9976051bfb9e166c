#!/bin/bash
# GP refit on device: parity tests, fit timing, per-phase timing (MPO_FIT_DEBUG), rocprof stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gp_fit_gpu.py tests/test_optimizer_gpu.py -x -v -s --timeout 120 \
    --timeout-method thread > gpurun_out/fit_tests.log 2>&1 && grep -E "device fit|passed|failed" gpurun_out/fit_tests.log && \
timeout -k 10 120 python -u scripts/fit_probe.py > gpurun_out/fit_probe.log 2>&1 && cat gpurun_out/fit_probe.log && \
for st in 1 2 3 4; do MPO_FIT_DEBUG=$st timeout -k 10 60 python -u scripts/fit_probe.py --reps 0 || exit 1; done && \
( cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/fitprof" -o fit \
    --output-format csv -- python "$GRAFT_REPO_ROOT/scripts/fit_probe.py" --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/fitprof.log" 2>&1 ) && \
cut -d, -f1-7 gpurun_out/fitprof/fit_kernel_stats.csv
