#!/bin/bash
# r06 session aj: MNIST conv2 weight-gradient buckets over two side streams (MPO_POP_PLAN wgs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/plan_ab.py --variants "wgs=1" "wgs=2" "wgs=1" "wgs=2" --trials 64 --rounds 4 --steps 4 > gpurun_out/aj_ab320.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "wgs=1" "wgs=2" --trials 8 --rounds 5 --steps 10 > gpurun_out/aj_ab40.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "wgs=1" "wgs=2" --trials 4 --rounds 5 --steps 10 > gpurun_out/aj_ab20.log 2>&1
