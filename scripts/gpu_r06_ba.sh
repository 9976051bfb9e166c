#!/bin/bash
# r06 session ba: the zero-bordered input gradient skips all-border tap rows per tile (MPO_POP_PLAN dgskip); k threshold re-swept
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py -k "formulations or side_stream or gradients" > gpurun_out/ba_tests.log 2>&1 && \
timeout -k 10 700 python -u scripts/plan_ab.py --variants "dgskip=0" "dgskip=1" "dgskip=1,dgfwd=6" "dgskip=1,dgfwd=8" "dgskip=1,dgfwd=10" "dgskip=1,dgfwd=7" "dgskip=0" "dgskip=1" --trials 64 --rounds 3 --steps 4 > gpurun_out/ba_ab320.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "dgskip=0" "dgskip=1,dgfwd=6" "dgskip=1,dgfwd=8" "dgskip=1,dgfwd=10" "dgskip=0" --trials 4 --rounds 4 --steps 10 > gpurun_out/ba_ab20.log 2>&1
