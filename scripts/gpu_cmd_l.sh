#!/bin/bash
# round 3, run l: LML host-staged direct IO -- GP fit / optimizer GPU suites, refit probe, rocprof of one refit at n = 256
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-l}
timeout -k 10 400 python -u -m pytest tests/test_gp_fit_gpu.py tests/test_optimizer_parity_gpu.py tests/test_optimizer_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_${T}.log 2>&1 && \
  tail -3 gpurun_out/tests_${T}.log && \
timeout -k 10 300 python -u scripts/refit_probe.py --n 64 128 256 512 > gpurun_out/refit_probe_${T}.log 2>&1 && cat gpurun_out/refit_probe_${T}.log && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/refit_probe.py --n 256 > /tmp/prof_${T}.log 2>&1 ) && \
mkdir -p gpurun_out/prof_refit256_${T} && find /tmp/prof_${T} -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_refit256_${T}/ \; && ls gpurun_out/prof_refit256_${T}
