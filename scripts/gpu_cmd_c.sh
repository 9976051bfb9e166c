cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/propose_probe.py > gpurun_out/propose_probe_c.log 2>&1 && cat gpurun_out/propose_probe_c.log && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_c -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/propose_probe.py > /tmp/prof_c.log 2>&1 ) && \
mkdir -p gpurun_out/prof_propose_c && find /tmp/prof_c -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_propose_c/ \; && \
timeout -k 10 500 python -u bench.py --workload search3 --no-pmc --no-cpu-baseline > gpurun_out/bench_search3_c.json 2> gpurun_out/bench_search3_c.err && cat gpurun_out/bench_search3_c.json
