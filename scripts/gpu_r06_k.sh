#!/bin/bash
# r06 session k: factor-broadcast sharded scoring tests + small-population diagnostics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gp_gpu.py::test_factor_copy_scores_bit_identical \
  tests/test_distributed_gpu.py::test_sharded_optimizer_scoring_matches_single_gpu \
  tests/test_search_gpu.py::test_configs3_layout_over_rccl_equals_one_process > gpurun_out/k_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/prof_variants.py j "xcd=4" "streams=1" --trials 4 > gpurun_out/j_prof20.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "xcd=4" "streams=1" "streams=2" "occmerge=1" "occmerge=0" --trials 4 --rounds 5 --steps 10 > gpurun_out/j_ab20.log 2>&1 && \
MPO_POP_PROFILE=1 timeout -k 10 200 python -u scripts/train_probe.py --trials 4 --steps 10 > gpurun_out/j_phase20.log 2>&1
