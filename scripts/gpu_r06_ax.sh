#!/bin/bash
# r06 session ax: DenseNet dn_wgrad3 chunk size (MPO_DN_PLAN wgpix)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/dn_ab.py --variants "wgpix=0" "wgpix=256" "wgpix=512" "wgpix=64" "wgpix=0" "wgpix=256" --rounds 4 --steps 5 > gpurun_out/ax_ab.log 2>&1 && \
MPO_DN_PLAN=wgpix=256 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_densenet_gpu.py > gpurun_out/ax_tests.log 2>&1
