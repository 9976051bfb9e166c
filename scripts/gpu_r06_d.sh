#!/bin/bash
# r06 session d: where the band input gradient's time goes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/prof_variants.py d "dgband=0" "dgband=1" "dgband=1,dgrmw=1" "dgband=1,dbg=8" "dgband=1,dbg=1" "dgband=0,dbg=1" > gpurun_out/d_prof.log 2>&1
