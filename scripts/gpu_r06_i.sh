#!/bin/bash
# r06 session i: occupancy / work-cut sweep of the conv2 input gradient and weight gradient
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/plan_ab.py --variants "dg_kb=78" "dg_kb=64" "dg_kb=52" "dg_kb=40" "dg_tiles=8,dg_kb=40" "dg_tiles=16" --rounds 5 --steps 4 > gpurun_out/i_dg_sweep.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "wg_spg2=2" "wg_spg2=1" "wg_spg2=4" "conv_kb1=52" "conv_kb2=78" --rounds 5 --steps 4 > gpurun_out/i_wg_sweep.log 2>&1
