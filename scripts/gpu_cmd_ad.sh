#!/bin/bash
# round 3: plan knob A/B (wgrad sample groups smaller, dgrad / conv LDS budgets)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ad}
timeout -k 10 500 python -u scripts/train_sweep.py base MPO_WG_SPG2=2 MPO_WG_SPG2=3 MPO_WG_SPG1=2 MPO_DG_KB=52 MPO_DG_KB=40 MPO_CONV_KB2=52 base > gpurun_out/train_sweep_${T}.log 2>&1; rc=$?; grep -A1 '^==' gpurun_out/train_sweep_${T}.log; exit $rc
