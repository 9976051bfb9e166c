#!/bin/bash
# r06 session as: conv2 weight gradient, a row pair of Ho = 2 (mod 4) pixels as one K run (MPO_POP_PLAN wgpair)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MPO_POP_PLAN=wgpair=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_trajectories_gpu.py > gpurun_out/as_tests.log 2>&1 && \
timeout -k 10 500 python -u scripts/plan_ab.py --variants "wgpair=0" "wgpair=1" "wgpair=0" "wgpair=1" --trials 64 --rounds 4 --steps 4 > gpurun_out/as_ab320.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "wgpair=0" "wgpair=1" "wgpair=0" "wgpair=1" --trials 4 --rounds 5 --steps 10 > gpurun_out/as_ab20.log 2>&1
