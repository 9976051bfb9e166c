#!/bin/bash
# r06 session ak: MNIST input-gradient buckets over three streams (MPO_POP_PLAN dgs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/plan_ab.py --variants "dgs=2" "dgs=3" "dgs=2" "dgs=3" --trials 64 --rounds 4 --steps 4 > gpurun_out/ak_ab320.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgs=2" "dgs=3" --trials 8 --rounds 5 --steps 10 > gpurun_out/ak_ab40.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgs=2" "dgs=3" --trials 4 --rounds 5 --steps 10 > gpurun_out/ak_ab20.log 2>&1
