#!/bin/bash
# r06 session j: where a small population's step goes (configs[0]: 4 trials x 5 folds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/prof_variants.py j "xcd=4" "streams=1" --trials 4 > gpurun_out/j_prof20.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "xcd=4" "streams=1" "streams=2" "occmerge=1" "occmerge=0" --trials 4 --rounds 5 --steps 10 > gpurun_out/j_ab20.log 2>&1 && \
MPO_POP_PROFILE=1 timeout -k 10 200 python -u scripts/train_probe.py --trials 4 --steps 10 > gpurun_out/j_phase20.log 2>&1
