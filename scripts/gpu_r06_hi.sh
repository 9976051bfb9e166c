#!/bin/bash
# r06 session hi: A/B of work-cut knobs (bits + time), then the default bench line and
# rocprofv3 kernel stats of its EI and train legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof_h_ei gpurun_out/prof_h_train
export TMPDIR=/tmp
R=$PWD
timeout -k 10 400 python -u scripts/plan_ab.py --variants "wgrpb=1" "wgrpb=2" "dg_kb=64" "dg_kb=52" "dg_kb=40" "dg_tiles=16" --rounds 5 --steps 4 > gpurun_out/i_sweep_320.log 2>&1 && \
timeout -k 10 300 python -u scripts/plan_ab.py --variants "wgrpb=1" "wgrpb=2" "dg_kb=52" --rounds 5 --steps 8 --shard 0/8 > gpurun_out/i_sweep_40.log 2>&1 && \
timeout -k 10 1000 python -u bench.py > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_h_ei -o run --output-format csv -- python -u $R/bench.py --workload ei --no-pmc --no-cpu-baseline > $R/gpurun_out/prof_h_ei/bench.json 2> $R/gpurun_out/prof_h_ei/bench.err ) && \
python -c "import glob,shutil; [shutil.copy(f, '$R/gpurun_out/prof_h_ei/') for f in glob.glob('/tmp/prof_h_ei/**/*_stats.csv', recursive=True)]" && \
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_h_train -o run --output-format csv -- python -u $R/bench.py --workload train --no-pmc --no-cpu-baseline > $R/gpurun_out/prof_h_train/bench.json 2> $R/gpurun_out/prof_h_train/bench.err ) && \
python -c "import glob,shutil; [shutil.copy(f, '$R/gpurun_out/prof_h_train/') for f in glob.glob('/tmp/prof_h_train/**/*_stats.csv', recursive=True)]"
