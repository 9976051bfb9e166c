#!/bin/bash
# r06 session aw: MNIST conv_kb1 / wg_spg2 follow-up (320, 40, 20 members)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u scripts/plan_ab.py --variants "xcd=4" "conv_kb1=30" "conv_kb1=24" "conv_kb1=36" "wg_spg2=3" "wg_spg2=4" "conv_kb1=30,wg_spg2=3" "conv_kb1=30,conv_kb2=120" "xcd=4" "conv_kb1=30" "conv_kb1=30,wg_spg2=3" --trials 64 --rounds 3 --steps 4 > gpurun_out/aw_ab320.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "xcd=4" "conv_kb1=30" "wg_spg2=3" "conv_kb1=30,wg_spg2=3" "xcd=4" --trials 8 --rounds 4 --steps 10 > gpurun_out/aw_ab40.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "xcd=4" "conv_kb1=30" "wg_spg2=3" "conv_kb1=30,wg_spg2=3" "xcd=4" --trials 4 --rounds 4 --steps 10 > gpurun_out/aw_ab20.log 2>&1
