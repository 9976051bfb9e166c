#!/bin/bash
# round 3: how much of conv2 fwd / dgrad is the weight-fragment fetch (MPO_POP_DEBUG=4: fragments from groups 0-1 only)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-af}
timeout -k 10 300 python -u scripts/train_sweep.py base MPO_POP_DEBUG=4 MPO_POP_DEBUG=1 base > gpurun_out/train_sweep_${T}.log 2>&1; rc=$?; grep -A1 '^==' gpurun_out/train_sweep_${T}.log; exit $rc
