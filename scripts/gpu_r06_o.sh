#!/bin/bash
# r06 session o: the look-ahead pivot sweep (MPO_FIT_LOOKAHEAD) -- bits, round time, lone chain, fit tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MPO_FIT_LOOKAHEAD=0 timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/la0.npz > gpurun_out/o_bits.log 2>&1 && \
MPO_FIT_LOOKAHEAD=1 timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/la1.npz /tmp/la0.npz >> gpurun_out/o_bits.log 2>&1 && \
for la in 0 1 0 1; do
  echo "== lookahead $la" >> gpurun_out/o_round.log
  MPO_FIT_LOOKAHEAD=$la timeout -k 10 120 python -u scripts/lml_round_prof.py 96 288 448 >> gpurun_out/o_round.log 2>&1 || exit 1
done && \
MPO_FIT_LOOKAHEAD=1 MPO_FIT_DEBUG=24 timeout -k 10 120 python -u scripts/step_stamps_probe.py 288 448 > gpurun_out/o_stamps.log 2>&1 && \
for la in 0 1; do
  echo "== lookahead $la" >> gpurun_out/o_chain.log
  MPO_FIT_LOOKAHEAD=$la timeout -k 10 200 python -u scripts/ask_chain_probe.py --ask-n 64 --reps 2 >> gpurun_out/o_chain.log 2>&1 || exit 1
done && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gp_fit_gpu.py > gpurun_out/o_tests.log 2>&1
