#!/bin/bash
# r06 session bf: samples per slab for the big members, 4 vs 5 / 6 / 8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u scripts/plan_ab.py --variants "xcd=4" "wg_spg2_big=5" "wg_spg2_big=6" "wg_spg2_big=8" "wg_spg2_big=6,wg_big=4" "xcd=4" --trials 64 --rounds 3 --steps 4 > gpurun_out/bf_ab320.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "xcd=4" "wg_spg2_big=5" "wg_spg2_big=6" "wg_spg2_big=8" "xcd=4" --trials 8 --rounds 4 --steps 10 > gpurun_out/bf_ab40.log 2>&1
