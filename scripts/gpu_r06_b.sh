#!/bin/bash
# r06 session b: band-form dgrad v2 (grouped K loop): correctness, A/B, kernel stats; G2 at n=200
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py tests/test_trajectories_gpu.py -q --timeout 200 --timeout-method thread > gpurun_out/tests_b_train.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/tests_b_train.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgband=0" "dgband=1" --rounds 6 --steps 4 > gpurun_out/dgband2_ab_320.log 2>&1 && \
timeout -k 10 200 python -u scripts/plan_ab.py --variants "dgband=0" "dgband=1" --rounds 6 --steps 8 --shard 0/8 > gpurun_out/dgband2_ab_40.log 2>&1 && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_b -o run -- python -u $GRAFT_REPO_ROOT/scripts/plan_ab.py --variants "dgband=0" "dgband=1" --rounds 2 --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_b.log 2>&1 ) && \
mkdir -p gpurun_out/prof_b && cp $(find /tmp/prof_b -name "*kernel_stats.csv") gpurun_out/prof_b/ ; \
timeout -k 10 400 python -u -m pytest tests/test_optimizer_parity_gpu.py tests/test_gp_fit_gpu.py -q --timeout 300 --timeout-method thread -s > gpurun_out/tests_b_g2.log 2>&1
echo "g2 rc=$?" >> gpurun_out/tests_b_g2.log
