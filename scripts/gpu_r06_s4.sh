#!/bin/bash
# r06: the configs[3] search in full on one GPU, final library (dgfwd, wgpair, conv_kb1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1150 python -u scripts/search_run.py gpurun_out/search3_full_r06b.json --world-size 129 --block-size 2 \
    --n-fold 5 --num-iterations 256 --epochs 10 --population-chunks 2 --n-samples 60000 --synthetic-labels learnable \
    > gpurun_out/search3_full_r06b.log 2>&1
