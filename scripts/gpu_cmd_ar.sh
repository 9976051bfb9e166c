#!/bin/bash
# round 3: pool_bwd with 4 elements' loads in flight per thread -- timing + training parity
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ar}
timeout -k 10 300 python -u scripts/train_sweep.py base base > gpurun_out/train_sweep_${T}.log 2>&1 && grep -A1 '^==' gpurun_out/train_sweep_${T}.log && \
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_trajectories_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_${T}.log 2>&1; rc=$?; tail -3 gpurun_out/tests_${T}.log; exit $rc
