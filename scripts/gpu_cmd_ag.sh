#!/bin/bash
# round 3: batched conv staging (stage_rows, 8 loads in flight per thread) -- timing + training parity tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ag}
timeout -k 10 300 python -u scripts/train_sweep.py base MPO_POP_DEBUG=1 base > gpurun_out/train_sweep_${T}.log 2>&1 && grep -A1 '^==' gpurun_out/train_sweep_${T}.log && \
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_trajectories_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_${T}.log 2>&1; rc=$?; tail -4 gpurun_out/tests_${T}.log; exit $rc
