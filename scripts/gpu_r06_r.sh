#!/bin/bash
# r06 session r: look-ahead workgroup first, X prefetch in the build, against the round-6 start library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=ab_libs/base/libmpo.so
MPO_LIB_AB=$B timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/base.npz > gpurun_out/r_bits.log 2>&1 && \
timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/cur.npz /tmp/base.npz >> gpurun_out/r_bits.log 2>&1 && \
MPO_FIT_LOOKAHEAD=0 timeout -k 10 120 python -u scripts/lml_bits_probe.py /tmp/cur0.npz /tmp/base.npz >> gpurun_out/r_bits.log 2>&1 && \
for v in base cur base cur kern; do
  echo "== $v" >> gpurun_out/r_round.log
  if [ $v = base ]; then MPO_LIB_AB=$B timeout -k 10 120 python -u scripts/lml_round_prof.py 96 288 448 >> gpurun_out/r_round.log 2>&1 || exit 1
  elif [ $v = kern ]; then HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python -u scripts/lml_round_prof.py 96 288 448 >> gpurun_out/r_round.log 2>&1 || exit 1
  else timeout -k 10 120 python -u scripts/lml_round_prof.py 96 288 448 >> gpurun_out/r_round.log 2>&1 || exit 1; fi
done && \
( cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace -d /tmp/r_tr -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/scripts/lml_round_prof.py" 288 > "$GRAFT_REPO_ROOT/gpurun_out/r_roundtr.log" 2>&1 ) && \
python3 scripts/lml_round_gaps.py "$(find /tmp/r_tr -name '*kernel_trace.csv' | head -1)" sw_xs_build > gpurun_out/r_gaps.log 2>&1 && \
for v in base cur; do
  echo "== $v" >> gpurun_out/r_chain.log
  if [ $v = base ]; then MPO_LIB_AB=$B timeout -k 10 200 python -u scripts/ask_chain_probe.py --ask-n 64 --reps 2 >> gpurun_out/r_chain.log 2>&1 || exit 1
  else timeout -k 10 200 python -u scripts/ask_chain_probe.py --ask-n 64 --reps 2 >> gpurun_out/r_chain.log 2>&1 || exit 1; fi
done && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gp_fit_gpu.py tests/test_optimizer_gpu.py > gpurun_out/r_tests.log 2>&1
