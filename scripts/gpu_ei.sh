#!/bin/bash
# EI kernel iteration: GP parity tests, then the EI bench leg (+ rocprof stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ei}
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gp_gpu.py tests/test_optimizer_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/ei_tests_$TAG.log 2>&1 && tail -2 gpurun_out/ei_tests_$TAG.log && \
timeout -k 10 300 python -u bench.py --workload ei --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_EXTRA:---no-pmc} \
    > gpurun_out/ei_bench_$TAG.json 2> gpurun_out/ei_bench_$TAG.err && cat gpurun_out/ei_bench_$TAG.json && \
( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG -o run --output-format csv -- \
    python "$GRAFT_REPO_ROOT/bench.py" --workload ei --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/ei_prof_$TAG.log" 2>&1 ) && \
mkdir -p gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$TAG/ \; && \
grep -h "gp_score" gpurun_out/prof_$TAG/*kernel_stats.csv
