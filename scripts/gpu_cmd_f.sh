#!/bin/bash
# round 3, run f: full -m gpu suite + smoke, GP probes (16-wave acq_grad), rocprof kernel stats of one refit at n = 256
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_f.log 2>&1 && \
  tail -3 gpurun_out/tests_f.log && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_f.log 2>&1 && cat gpurun_out/smoke_f.log && \
timeout -k 10 300 python -u scripts/propose_probe.py > gpurun_out/propose_probe_f.log 2>&1 && cat gpurun_out/propose_probe_f.log && \
timeout -k 10 300 python -u scripts/refit_probe.py --n 64 128 256 512 > gpurun_out/refit_probe_f.log 2>&1 && cat gpurun_out/refit_probe_f.log && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_f -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/refit_probe.py --n 256 > /tmp/prof_f.log 2>&1 ) && \
mkdir -p gpurun_out/prof_refit256_f && find /tmp/prof_f -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_refit256_f/ \; && ls gpurun_out/prof_refit256_f
