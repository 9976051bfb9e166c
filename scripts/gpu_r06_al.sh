#!/bin/bash
# r06 session al: the stream variants on the bench's 8-GPU share (LPT share 0 of 8 of the 320 members)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/plan_ab.py --variants "wgs=1,dgs=2" "wgs=2,dgs=3" "wgs=1,dgs=3" "wgs=2,dgs=2" --trials 64 --shard 0/8 --rounds 6 --steps 10 > gpurun_out/al_shard.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "wgs=1,dgs=2" "wgs=2,dgs=3" --trials 64 --shard 3/8 --rounds 6 --steps 10 > gpurun_out/al_shard3.log 2>&1
