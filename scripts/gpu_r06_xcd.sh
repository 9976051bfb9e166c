#!/bin/bash
# r06: XCD-run item order A/B (timing, bits, HBM traffic)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/plan_ab.py --variants "xcd=0" "xcd=2" "xcd=4" "xcd=8" "xcd=16" "xcd=32" --rounds 6 --steps 4 > gpurun_out/xcd2_ab_320.log 2>&1 && \
timeout -k 10 200 python -u scripts/plan_ab.py --variants "xcd=0" "xcd=2" "xcd=4" "xcd=8" "xcd=16" "xcd=32" --rounds 6 --steps 8 --shard 0/8 > gpurun_out/xcd2_ab_40.log 2>&1 && \
timeout -k 10 900 python -u scripts/train_pmc_ab.py "xcd=0" "xcd=4" "xcd=16" > gpurun_out/xcd2_pmc.log 2>&1
