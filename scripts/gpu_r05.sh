#!/bin/bash
# One GPU session (round 5).  Every GPU step has its own time limit; steps are
# chained with && so the first failure (fault, abort, time limit) ends the script.
#   TESTS=<pytest paths|none>  TEST_TIMEOUT=<s>  PROBES=<python commands separated by ';;'>
#   BENCH=0|1  BENCH_ARGS=<args>  PROF=1  TAG=<suffix>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05}
TESTS=${TESTS:-tests}
step_tests() {
  [ "$TESTS" = "none" ] && return 0
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread \
      > gpurun_out/gpu_tests_$TAG.log 2>&1 && echo "TESTS OK" && tail -3 gpurun_out/gpu_tests_$TAG.log
}
step_smoke() {
  [ "${SMOKE:-0}" = "0" ] && return 0
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
      cat gpurun_out/smoke_$TAG.log
}
step_probes() {
  [ -z "$PROBES" ] && return 0
  local i=0
  local IFS_OLD="$IFS"
  while IFS= read -r cmd; do
    [ -z "$cmd" ] && continue
    i=$((i+1))
    echo "== probe $i: $cmd"
    timeout -k 10 ${PROBE_TIMEOUT:-600} $cmd > gpurun_out/probe_${TAG}_$i.log 2>&1 || { echo "probe $i failed"; tail -20 gpurun_out/probe_${TAG}_$i.log; return 1; }
    tail -${PROBE_TAIL:-12} gpurun_out/probe_${TAG}_$i.log
  done < <(echo "$PROBES" | sed 's/;;/\n/g')
  IFS="$IFS_OLD"
}
step_bench() {
  [ "${BENCH:-0}" = "0" ] && return 0
  timeout -k 10 ${BENCH_TIMEOUT:-900} python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 3} \
      > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json
}
step_prof() {
  [ "${PROF:-0}" = "0" ] && return 0
  ( cd /tmp && rm -rf /tmp/prof_$TAG && timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d /tmp/prof_$TAG \
      -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" ${PROF_ARGS:---steps 10 --warmup 2 --no-cpu-baseline --no-pmc} \
      > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 ) && \
  mkdir -p gpurun_out/prof_$TAG && find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_$TAG/ \; && \
  echo "PROF OK" && ls gpurun_out/prof_$TAG
}
step_tests && step_smoke && step_probes && step_bench && step_prof
