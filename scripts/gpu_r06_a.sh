#!/bin/bash
# r06 session a: GPU tests with the band-form input gradient, then its A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_a.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/tests_a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/plan_ab.py --variants "dgband=0" "dgband=1" "dgband=1,xcd=4" --rounds 6 --steps 4 > gpurun_out/dgband_ab_320.log 2>&1 && \
timeout -k 10 200 python -u scripts/plan_ab.py --variants "dgband=0" "dgband=1" "dgband=1,xcd=4" --rounds 6 --steps 8 --shard 0/8 > gpurun_out/dgband_ab_40.log 2>&1
