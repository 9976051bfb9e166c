#!/bin/bash
# r06 session bc: more samples per conv2 weight-gradient slab for the members with many m-groups (MPO_POP_PLAN wg_spg2_big / wg_big)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u scripts/plan_ab.py --variants "xcd=4" "wg_spg2_big=4" "wg_spg2_big=4,wg_big=2" "wg_spg2_big=4,wg_big=5" "wg_spg2_big=3" "xcd=4" "wg_spg2_big=4" --trials 64 --rounds 3 --steps 4 > gpurun_out/bc_ab320.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "xcd=4" "wg_spg2_big=4" "wg_spg2_big=4,wg_big=2" "wg_spg2_big=4,wg_big=5" "xcd=4" --trials 8 --rounds 4 --steps 10 > gpurun_out/bc_ab40.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "xcd=4" "wg_spg2_big=4" "wg_spg2_big=4,wg_big=2" "wg_spg2_big=4,wg_big=5" "xcd=4" --trials 4 --rounds 4 --steps 10 > gpurun_out/bc_ab20.log 2>&1
