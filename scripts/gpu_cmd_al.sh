#!/bin/bash
# round 3: forward conv with up to 4 m-tiles per wave (MPO_CONV_MT=4: items of up to 256 pixels) -- A/B + parity
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-al}
timeout -k 10 400 python -u scripts/train_sweep.py base MPO_CONV_MT=4 MPO_CONV_MT=4,MPO_CONV_KB2=100 MPO_CONV_MT=4,MPO_CONV_KB1=40,MPO_CONV_KB2=52 base > gpurun_out/train_sweep_${T}.log 2>&1 && grep -A1 '^==' gpurun_out/train_sweep_${T}.log && \
MPO_CONV_MT=4 timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_${T}.log 2>&1; rc=$?; tail -3 gpurun_out/tests_${T}.log; exit $rc
