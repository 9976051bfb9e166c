#!/bin/bash
# One GPU session (round 3): parity tests, smoke, probes, bench, rocprof kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the first
# failure (fault, abort, time limit) ends the script.
#   TESTS=<pytest paths|none>  TEST_TIMEOUT=<s>  PROBE=<python command|empty>  BENCH=0|1
#   BENCH_ARGS=<args>  PROF=1  TAG=<suffix>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
TESTS=${TESTS:-tests}
step_tests() {
  [ "$TESTS" = "none" ] && return 0
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread \
      > gpurun_out/gpu_tests_$TAG.log 2>&1 && echo "TESTS OK" && tail -3 gpurun_out/gpu_tests_$TAG.log
}
step_smoke() {
  [ "${SMOKE:-1}" = "0" ] && return 0
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
      cat gpurun_out/smoke_$TAG.log
}
step_probe() {
  [ -z "$PROBE" ] && return 0
  timeout -k 10 ${PROBE_TIMEOUT:-300} $PROBE > gpurun_out/probe_$TAG.log 2>&1 && cat gpurun_out/probe_$TAG.log
}
step_bench() {
  [ "${BENCH:-1}" = "0" ] && return 0
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 3} \
      > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json
}
step_prof() {
  [ "${PROF:-0}" = "0" ] && return 0
  # traces stay on the box (/tmp): only the kernel-stats summary comes back
  ( cd /tmp && rm -rf /tmp/prof_$TAG && timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG \
      -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" ${PROF_ARGS:---steps 10 --warmup 2 --no-cpu-baseline --no-pmc} \
      > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 ) && \
  mkdir -p gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$TAG/ \; && \
  echo "PROF OK" && ls gpurun_out/prof_$TAG
}
step_tests && step_smoke && step_probe && step_bench && step_prof
