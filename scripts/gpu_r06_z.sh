#!/bin/bash
# r06 session z: the default bench line after dgfwd + DenseNet bnfuse + rocprofv3 kernel stats of its EI and train legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof_z_ei gpurun_out/prof_z_train
export TMPDIR=/tmp
R=$PWD
timeout -k 10 1000 python -u bench.py > gpurun_out/bench_z.json 2> gpurun_out/bench_z.err && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_z_ei -o run --output-format csv -- python -u $R/bench.py --workload ei --no-pmc --no-cpu-baseline > $R/gpurun_out/prof_z_ei/bench.json 2> $R/gpurun_out/prof_z_ei/bench.err ) && \
python -c "import glob,shutil; [shutil.copy(f, '$R/gpurun_out/prof_z_ei/') for f in glob.glob('/tmp/prof_z_ei/**/*_stats.csv', recursive=True)]" && \
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_z_train -o run --output-format csv -- python -u $R/bench.py --workload train --no-pmc --no-cpu-baseline > $R/gpurun_out/prof_z_train/bench.json 2> $R/gpurun_out/prof_z_train/bench.err ) && \
python -c "import glob,shutil; [shutil.copy(f, '$R/gpurun_out/prof_z_train/') for f in glob.glob('/tmp/prof_z_train/**/*_stats.csv', recursive=True)]"
