#!/bin/bash
# round 3: wgrad sample-group size A/B (partial slab count vs parallelism)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ac}
timeout -k 10 500 python -u scripts/train_sweep.py base MPO_WG_SPG2=8 MPO_WG_SPG2=12 MPO_WG_SPG2=20 MPO_WG_SPG2=8,MPO_WG_SPG1=10 MPO_WG_SPG1=10 base > gpurun_out/train_sweep_${T}.log 2>&1; rc=$?; cat gpurun_out/train_sweep_${T}.log; exit $rc
