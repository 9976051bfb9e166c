#!/bin/bash
# r06 session ab: the refit round replayed from a hipGraph (MPO_FIT_GRAPH) -- lone chain, turnaround, fit tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 0 1 0 1; do
  echo "== graph $g" >> gpurun_out/ab_chain.log
  MPO_FIT_GRAPH=$g timeout -k 10 200 python -u scripts/ask_chain_probe.py --ask-n 64 --reps 2 >> gpurun_out/ab_chain.log 2>&1 || exit 1
done && \
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/ab_tr -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/scripts/ask_chain_probe.py" --ask-n 16 --reps 1 > "$GRAFT_REPO_ROOT/gpurun_out/ab_chain_tr.log" 2>&1 ) && \
python3 scripts/chain_gaps.py "$(find /tmp/ab_tr -name '*kernel_trace.csv' | head -1)" > gpurun_out/ab_gaps.log 2>&1 && \
python3 scripts/lml_round_gaps.py "$(find /tmp/ab_tr -name '*kernel_trace.csv' | head -1)" sw_xs_build >> gpurun_out/ab_gaps.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gp_fit_gpu.py tests/test_optimizer_gpu.py tests/test_optimizer_parity_gpu.py > gpurun_out/ab_tests.log 2>&1
