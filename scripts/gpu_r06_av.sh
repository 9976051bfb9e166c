#!/bin/bash
# r06 session av: MNIST plan knobs re-swept after dgfwd + wgpair (320 members, then 40)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u scripts/plan_ab.py --variants "xcd=4" "dg_tiles=8" "dg_tiles=16" "dg_kb=100" "conv_kb1=52" "conv_kb1=30" "conv_kb2=78" "wg_spg2=3" "wg_spg2=1" "dgf_kb1=120" "conv_mt=2" "xcd=4" --trials 64 --rounds 3 --steps 4 > gpurun_out/av_ab320.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "xcd=4" "dg_tiles=8" "dg_tiles=16" "conv_kb1=52" "wg_spg2=1" "conv_mt=2" "xcd=4" --trials 8 --rounds 4 --steps 10 > gpurun_out/av_ab40.log 2>&1
