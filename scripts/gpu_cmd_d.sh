#!/bin/bash
# round 3, run d: blocked prepare factorisation -- GP parity tests first, then the probes and the search3 leg
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gp_gpu.py tests/test_optimizer_gpu.py tests/test_optimizer_parity_gpu.py \
    tests/test_gp_fit_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gp_tests_d.log 2>&1 && \
  tail -3 gpurun_out/gp_tests_d.log && \
timeout -k 10 300 python -u scripts/propose_probe.py > gpurun_out/propose_probe_d.log 2>&1 && cat gpurun_out/propose_probe_d.log && \
timeout -k 10 300 python -u scripts/refit_probe.py --n 64 128 256 512 > gpurun_out/refit_probe_d.log 2>&1 && cat gpurun_out/refit_probe_d.log && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_d -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/propose_probe.py > /tmp/prof_d.log 2>&1 ) && \
mkdir -p gpurun_out/prof_propose_d && find /tmp/prof_d -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_propose_d/ \; && \
timeout -k 10 600 python -u bench.py --workload search3 --no-pmc --no-cpu-baseline > gpurun_out/bench_search3_d.json 2> gpurun_out/bench_search3_d.err && cat gpurun_out/bench_search3_d.json
