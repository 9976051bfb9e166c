#!/bin/bash
# r06 session bb: bit-neutral MNIST plan knobs re-swept on the final plan (320 and 40 members)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u scripts/plan_ab.py --variants "xcd=4" "xcd=2" "xcd=8" "occmerge=0" "occfill=2" "occfill=8" "dgs=2" "wgs=1" "dg_tiles=14" "dg_kb=64" "xcd=4" --trials 64 --rounds 3 --steps 4 > gpurun_out/bb_ab320.log 2>&1 && \
timeout -k 10 400 python -u scripts/plan_ab.py --variants "xcd=4" "xcd=2" "xcd=8" "occfill=2" "occfill=8" "dg_tiles=14" "xcd=4" --trials 8 --rounds 4 --steps 10 > gpurun_out/bb_ab40.log 2>&1
