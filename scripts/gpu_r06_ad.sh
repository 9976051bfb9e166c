#!/bin/bash
# r06 session ad/ae: sw_pairs_final_kernel with staged operands -- bits against the round-6 start library, timeline, lone chain, fit tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
MPO_LIB_AB=ab_libs/base/libmpo.so timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/base.npz > gpurun_out/ae_bits.log 2>&1 && timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/cur.npz /tmp/base.npz >> gpurun_out/ae_bits.log 2>&1 && MPO_FIT_DEBUG=25 timeout -k 10 120 python -u scripts/pair_stamps_probe.py 96 288 448 > gpurun_out/ae_pairs.log 2>&1 && for i in 1 2; do timeout -k 10 200 python -u scripts/ask_chain_probe.py --ask-n 64 --reps 1 >> gpurun_out/ae_chain.log 2>&1 || exit 1; done && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gp_fit_gpu.py > gpurun_out/ae_tests.log 2>&1
