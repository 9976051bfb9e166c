#!/bin/bash
# r06 session aq: forward-formulation input gradient on by default (k <= 4, 80 KiB budget): tests + A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_trajectories_gpu.py > gpurun_out/aq_tests.log 2>&1 && \
timeout -k 10 500 python -u scripts/plan_ab.py --variants "dgfwd=0" "dgfwd=4" "dgfwd=0" "dgfwd=4" --trials 64 --rounds 4 --steps 4 > gpurun_out/aq_ab320.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgfwd=0" "dgfwd=4" "dgfwd=0" "dgfwd=4" --trials 8 --rounds 5 --steps 10 > gpurun_out/aq_ab40.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgfwd=0" "dgfwd=4" "dgfwd=0" "dgfwd=4" --trials 4 --rounds 5 --steps 10 > gpurun_out/aq_ab20.log 2>&1
