#!/bin/bash
# r06 session ap: which k take the forward-formulation input gradient (MPO_POP_PLAN dgfset mask), LDS budget
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/plan_ab.py --variants "dgfwd=0" "dgfset=16" "dgfset=48" "dgfset=80" "dgfset=144" "dgfset=272" "dgfset=528" "dgfset=1040" "dgfset=16,dgf_kb1=80" "dgfset=16,dgf_kb1=110" "dgfset=16,dgf_kb1=160" "dgfwd=0" --trials 64 --rounds 4 --steps 4 > gpurun_out/ap_ab320.log 2>&1
