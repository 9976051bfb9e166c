#!/bin/bash
# round 3: conv2 input-gradient tiles per work item A/B
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ap}
timeout -k 10 400 python -u scripts/train_sweep.py base MPO_DG_TILES=8 MPO_DG_TILES=12 base > gpurun_out/train_sweep_${T}.log 2>&1; rc=$?; grep '^==' gpurun_out/train_sweep_${T}.log; grep -o 'conv2_dgrad=[0-9.]*' gpurun_out/train_sweep_${T}.log | head; exit $rc
