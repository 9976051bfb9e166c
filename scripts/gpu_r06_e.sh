#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/prof_variants.py e "dgband=0" "dgband=1" "dgband=1,dgrmw=1" "dgband=1,dbg=8" "dgband=1,dbg=1" > gpurun_out/e_prof.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgband=0" "dgband=1" "dgband=1,dgrmw=1" --rounds 6 --steps 4 > gpurun_out/e_ab_320.log 2>&1
