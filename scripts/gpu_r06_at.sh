#!/bin/bash
# r06 session at: DenseNet split BN backward (scale dy in the conv epilogue, the affine part per segment; MPO_DN_PLAN bnsplit)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_densenet_gpu.py tests/test_trajectories_gpu.py > gpurun_out/at_tests.log 2>&1 && \
timeout -k 10 400 python -u scripts/dn_ab.py --variants "bnsplit=0" "bnsplit=1" "bnsplit=0" "bnsplit=1" --rounds 5 --steps 5 > gpurun_out/at_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/prof_variants.py at --dn "bnsplit=0" "bnsplit=1" > gpurun_out/at_prof.log 2>&1
