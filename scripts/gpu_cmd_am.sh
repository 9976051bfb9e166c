#!/bin/bash
# round 3: forward conv MT=4 LDS budget sweep
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-am}
timeout -k 10 500 python -u scripts/train_sweep.py base MPO_CONV_MT=4,MPO_CONV_KB1=32,MPO_CONV_KB2=40 MPO_CONV_MT=4,MPO_CONV_KB1=40,MPO_CONV_KB2=52 MPO_CONV_MT=4,MPO_CONV_KB1=52,MPO_CONV_KB2=100 MPO_CONV_MT=4,MPO_CONV_KB1=78,MPO_CONV_KB2=100 MPO_CONV_KB1=40,MPO_CONV_KB2=52 MPO_CONV_MT=4,MPO_CONV_KB1=40,MPO_CONV_KB2=100 > gpurun_out/train_sweep_${T}.log 2>&1; rc=$?; grep '^==' gpurun_out/train_sweep_${T}.log; grep -o 'conv2_fwd=[0-9.]*  conv1_wgrad=[0-9.]*  conv1_fwd=[0-9.]*\|conv2_fwd=[0-9.]*' gpurun_out/train_sweep_${T}.log | head -20; exit $rc
