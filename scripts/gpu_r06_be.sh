#!/bin/bash
# r06 session be: the whole GPU suite + smoke + bench on the final library (after wg_spg2_big)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof_be_ei gpurun_out/prof_be_train
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/be_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/be_smoke.log 2>&1 && \
timeout -k 10 700 python -u bench.py > gpurun_out/bench_be.json 2> gpurun_out/bench_be.err && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_be_ei -o run --output-format csv -- python -u $R/bench.py --workload ei --no-pmc --no-cpu-baseline > $R/gpurun_out/prof_be_ei/bench.json 2> $R/gpurun_out/prof_be_ei/bench.err ) && \
python -c "import glob,shutil; [shutil.copy(f, '$R/gpurun_out/prof_be_ei/') for f in glob.glob('/tmp/prof_be_ei/**/*_stats.csv', recursive=True)]" && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_be_train -o run --output-format csv -- python -u $R/bench.py --workload train --no-pmc --no-cpu-baseline > $R/gpurun_out/prof_be_train/bench.json 2> $R/gpurun_out/prof_be_train/bench.err ) && \
python -c "import glob,shutil; [shutil.copy(f, '$R/gpurun_out/prof_be_train/') for f in glob.glob('/tmp/prof_be_train/**/*_stats.csv', recursive=True)]"
