#!/bin/bash
# r06 session ao: dgfwd threshold and LDS budget of the forward-formulation input gradient
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/plan_ab.py --variants "dgfwd=0" "dgfwd=3" "dgfwd=4" "dgfwd=5" "dgfwd=4,dgf_kb1=60" "dgfwd=4,dgf_kb1=80" "dgfwd=5,dgf_kb1=80" "dgfwd=4,dgf_kb1=24,dgf_kb2=60" --trials 64 --rounds 4 --steps 4 > gpurun_out/ao_ab320.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgfwd=0" "dgfwd=4" "dgfwd=5" "dgfwd=6" "dgfwd=4,dgf_kb1=80" --trials 8 --rounds 5 --steps 10 > gpurun_out/ao_ab40.log 2>&1
