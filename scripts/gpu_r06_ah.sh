#!/bin/bash
# r06 session ah: DenseNet weight gradients on two side streams (MPO_DN_PLAN wg2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_densenet_gpu.py tests/test_trajectories_gpu.py > gpurun_out/ah_tests.log 2>&1 && \
timeout -k 10 400 python -u scripts/dn_ab.py --variants "wg2=0" "wg2=1" --rounds 5 --steps 5 > gpurun_out/ah_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/prof_variants.py ah --dn "wg2=0" "wg2=1" > gpurun_out/ah_prof.log 2>&1
