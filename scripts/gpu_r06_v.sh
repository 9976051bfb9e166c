#!/bin/bash
# r06 session v: the tiled K build (MPO_FIT_BUILD) -- bits against the round-6 start library, round time, chain
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=ab_libs/base/libmpo.so
MPO_LIB_AB=$B timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/base.npz > gpurun_out/v_bits.log 2>&1 && \
timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/cur.npz /tmp/base.npz >> gpurun_out/v_bits.log 2>&1 && \
MPO_FIT_BUILD=rows timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/rows.npz /tmp/base.npz >> gpurun_out/v_bits.log 2>&1 && \
for v in rows tile rows tile; do
  echo "== $v" >> gpurun_out/v_round.log
  if [ $v = rows ]; then MPO_FIT_BUILD=rows timeout -k 10 120 python -u scripts/lml_round_prof.py 96 288 448 >> gpurun_out/v_round.log 2>&1 || exit 1
  else timeout -k 10 120 python -u scripts/lml_round_prof.py 96 288 448 >> gpurun_out/v_round.log 2>&1 || exit 1; fi
done && \
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/v_tr -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/scripts/ask_chain_probe.py" --ask-n 16 --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/v_chain_tr.log" 2>&1 ) && \
python3 scripts/chain_gaps.py "$(find /tmp/v_tr -name '*kernel_trace.csv' | head -1)" > gpurun_out/v_gaps.log 2>&1 && \
python3 scripts/lml_round_gaps.py "$(find /tmp/v_tr -name '*kernel_trace.csv' | head -1)" sw_xs_build >> gpurun_out/v_gaps.log 2>&1 && \
for v in base cur; do
  echo "== $v" >> gpurun_out/v_chain.log
  if [ $v = base ]; then MPO_LIB_AB=$B timeout -k 10 200 python -u scripts/ask_chain_probe.py --ask-n 64 --reps 2 >> gpurun_out/v_chain.log 2>&1 || exit 1
  else timeout -k 10 200 python -u scripts/ask_chain_probe.py --ask-n 64 --reps 2 >> gpurun_out/v_chain.log 2>&1 || exit 1; fi
done && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gp_fit_gpu.py tests/test_optimizer_gpu.py > gpurun_out/v_tests.log 2>&1
