#!/bin/bash
# r06 session p: step workgroups of 2 / 4 / 8 waves (MPO_FIT_STEP_WAVES) with the look-ahead: sweep latency,
# bits, round time, lone chain
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./scripts/probes/sweep_lat > gpurun_out/p_sweep_lat.log 2>&1 && \
MPO_FIT_LOOKAHEAD=0 timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/ref.npz > gpurun_out/p_bits.log 2>&1 && \
for nw in 2 4 8; do
  MPO_FIT_STEP_WAVES=$nw timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/w$nw.npz /tmp/ref.npz >> gpurun_out/p_bits.log 2>&1 || exit 1
done && \
for nw in 4 8 2 4 8; do
  echo "== waves $nw" >> gpurun_out/p_round.log
  MPO_FIT_STEP_WAVES=$nw timeout -k 10 120 python -u scripts/lml_round_prof.py 96 288 448 >> gpurun_out/p_round.log 2>&1 || exit 1
done && \
for nw in 4 8; do
  echo "== waves $nw" >> gpurun_out/p_chain.log
  MPO_FIT_STEP_WAVES=$nw timeout -k 10 200 python -u scripts/ask_chain_probe.py --ask-n 64 --reps 2 >> gpurun_out/p_chain.log 2>&1 || exit 1
done
