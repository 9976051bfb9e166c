#!/bin/bash
# r06 session an: conv2 input gradient as a zero-bordered forward conv for small k (MPO_POP_PLAN dgfwd)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MPO_POP_PLAN=dgfwd=10 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_trajectories_gpu.py > gpurun_out/an_tests.log 2>&1 && \
timeout -k 10 500 python -u scripts/plan_ab.py --variants "dgfwd=0" "dgfwd=4" "dgfwd=6" "dgfwd=8" "dgfwd=10" "dgfwd=0" --trials 64 --rounds 4 --steps 4 > gpurun_out/an_ab320.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgfwd=0" "dgfwd=5" "dgfwd=7" "dgfwd=10" --trials 4 --rounds 5 --steps 10 > gpurun_out/an_ab20.log 2>&1 && \
timeout -k 10 400 python -u scripts/prof_variants.py an "dgfwd=0" "dgfwd=10" > gpurun_out/an_prof.log 2>&1
