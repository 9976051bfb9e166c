#!/bin/bash
# r06 session am: DenseNet BN backward reduce fused, on top of two weight-gradient streams (MPO_DN_PLAN bnfuse)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_densenet_gpu.py tests/test_trajectories_gpu.py > gpurun_out/am_tests.log 2>&1 && \
timeout -k 10 400 python -u scripts/dn_ab.py --variants "bnfuse=0" "bnfuse=1" "bnfuse=0" "bnfuse=1" --rounds 5 --steps 5 > gpurun_out/am_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/prof_variants.py am --dn "bnfuse=0" "bnfuse=1" > gpurun_out/am_prof.log 2>&1
