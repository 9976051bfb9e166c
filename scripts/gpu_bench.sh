#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
