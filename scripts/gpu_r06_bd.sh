#!/bin/bash
# r06 session bd: wg_spg2_big = 4 by default -- MNIST GPU tests (oracle parity, isolation, trajectories) + A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_trajectories_gpu.py tests/test_search_gpu.py > gpurun_out/bd_tests.log 2>&1 && \
timeout -k 10 500 python -u scripts/plan_ab.py --variants "wg_spg2_big=0" "wg_spg2_big=4" "wg_spg2_big=0" "wg_spg2_big=4" --trials 64 --rounds 3 --steps 4 > gpurun_out/bd_ab320.log 2>&1
