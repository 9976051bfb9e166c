#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel stats.  Each GPU step has
# its own time limit; steps are chained with && so a failure stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-420} python -u -m pytest $TESTS -m gpu -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 && echo "TESTS OK" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && cat gpurun_out/smoke.log && \
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cat gpurun_out/bench.json && \
( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o ei \
    --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline \
    > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 ) && echo "PROF OK"
