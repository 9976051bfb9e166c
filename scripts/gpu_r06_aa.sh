#!/bin/bash
# r06 session aa: conv2 weight gradient, DMA two pairs ahead for the small-F buckets (MPO_POP_PLAN wgdeep)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/plan_ab.py --variants "wgdeep=0" "wgdeep=1" "wgdeep=2" "wgdeep=4" --trials 64 --rounds 4 --steps 4 > gpurun_out/aa_ab320.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "wgdeep=0" "wgdeep=2" "wgdeep=4" --trials 4 --rounds 5 --steps 10 > gpurun_out/aa_ab20.log 2>&1 && \
timeout -k 10 400 python -u scripts/prof_variants.py aa "wgdeep=0" "wgdeep=2" "wgdeep=4" > gpurun_out/aa_prof.log 2>&1
