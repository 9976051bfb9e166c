#!/bin/bash
# scoring kernel: parity, then the in-process A/B of scripts/ei_ab.py (env-switch variants)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-var}
for v in default; do
  timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gp_gpu.py} -m gpu -q --timeout 120 --timeout-method thread \
      > gpurun_out/ei_tests_${TAG}_$v.log 2>&1; rc=$?
  tail -1 gpurun_out/ei_tests_${TAG}_$v.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
  timeout -k 10 200 python -u scripts/ei_ab.py ${AB_ARGS:-occ4=MPO_GP_OCC:4 occ5=MPO_GP_OCC:5 occ6=MPO_GP_OCC:6} 2>&1 | grep -v amdgpu.ids || exit 1
done
