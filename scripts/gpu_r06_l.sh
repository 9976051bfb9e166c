#!/bin/bash
# r06 session l: the pivot sweep with 4 steps per LDS round (MPO_FIT_SWEEP_STEPS) vs 2:
# bits, LML round time, a lone cl_min chain
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MPO_FIT_SWEEP_STEPS=2 timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/s2.npz > gpurun_out/l_bits.log 2>&1 && \
MPO_FIT_SWEEP_STEPS=4 timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/s4.npz /tmp/s2.npz >> gpurun_out/l_bits.log 2>&1 && \
for st in 2 4 2 4; do
  echo "== steps $st" >> gpurun_out/l_round.log
  MPO_FIT_SWEEP_STEPS=$st timeout -k 10 120 python -u scripts/lml_round_prof.py 96 256 448 >> gpurun_out/l_round.log 2>&1 || exit 1
done && \
for st in 2 4; do
  echo "== steps $st" >> gpurun_out/l_chain.log
  MPO_FIT_SWEEP_STEPS=$st timeout -k 10 200 python -u scripts/ask_chain_probe.py --ask-n 64 --reps 2 >> gpurun_out/l_chain.log 2>&1 || exit 1
done
