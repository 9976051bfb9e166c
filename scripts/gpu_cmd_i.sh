#!/bin/bash
# round 3, run i: fused EI finish -- GP / optimizer GPU suites, smoke, EI bench leg with live PMC traffic, rocprof kernel stats of the EI leg
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-i}
timeout -k 10 400 python -u -m pytest tests/test_gp_gpu.py tests/test_optimizer_gpu.py tests/test_optimizer_parity_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_${T}.log 2>&1 && \
  tail -3 gpurun_out/tests_${T}.log && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${T}.log 2>&1 && cat gpurun_out/smoke_${T}.log && \
timeout -k 10 400 python -u bench.py --workload ei --steps 20 --warmup 5 > gpurun_out/bench_ei_${T}.json 2> gpurun_out/bench_ei_${T}.err && cat gpurun_out/bench_ei_${T}.json && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload ei --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > /tmp/prof_${T}.log 2>&1 ) && \
mkdir -p gpurun_out/prof_ei_${T} && find /tmp/prof_${T} -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_ei_${T}/ \; && ls gpurun_out/prof_ei_${T}
