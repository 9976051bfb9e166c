#!/bin/bash
# r06 session c: band dgrad v3 (unconditional prefetch) + gather dgrad with unconditional prefetch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgband=0" "dgband=0,dgpf=1" "dgband=1" --rounds 6 --steps 4 > gpurun_out/c_ab_320.log 2>&1 && \
timeout -k 10 200 python -u scripts/plan_ab.py --variants "dgband=0" "dgband=0,dgpf=1" "dgband=1" --rounds 6 --steps 8 --shard 0/8 > gpurun_out/c_ab_40.log 2>&1 && \
timeout -k 10 600 python -u scripts/prof_variants.py c "dgband=0" "dgband=0,dgpf=1" "dgband=1" > gpurun_out/c_prof.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py tests/test_trajectories_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/c_tests_train.log 2>&1
echo "rc=$?" >> gpurun_out/c_tests_train.log
