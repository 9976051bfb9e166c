#!/bin/bash
# r06 session ai: DenseNet weight gradients on three side streams (MPO_DN_PLAN wgs=3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_densenet_gpu.py tests/test_trajectories_gpu.py > gpurun_out/ai_tests.log 2>&1 && \
timeout -k 10 400 python -u scripts/dn_ab.py --variants "wg2=1" "wg2=1,wgs=3" --rounds 5 --steps 5 > gpurun_out/ai_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/prof_variants.py ai --dn "wg2=1" "wg2=1,wgs=3" > gpurun_out/ai_prof.log 2>&1
