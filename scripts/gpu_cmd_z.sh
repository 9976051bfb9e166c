#!/bin/bash
# round 3, run z: host-direct polish objective (mpo_gp_acq_grad_host) -- GP / optimizer GPU suites, proposal probe,
# then rocprofv3 kernel stats of the bench's ei, fit, train and densenet legs
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-z}
timeout -k 10 400 python -u -m pytest tests/test_gp_gpu.py tests/test_optimizer_gpu.py tests/test_optimizer_parity_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_${T}.log 2>&1 && \
  tail -3 gpurun_out/tests_${T}.log && \
timeout -k 10 300 python -u scripts/propose_probe.py > gpurun_out/propose_probe_${T}.log 2>&1 && cat gpurun_out/propose_probe_${T}.log && \
for W in ei fit train densenet; do
  ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T}_$W -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_$W.log 2>&1 ) || exit 1
  mkdir -p gpurun_out/prof_${T}_$W && find /tmp/prof_${T}_$W -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_${T}_$W/ \;
done && ls gpurun_out/prof_${T}_*
