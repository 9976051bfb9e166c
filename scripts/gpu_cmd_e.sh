#!/bin/bash
# round 3, run e: GP + training parity tests, GP probes, XCD-order A/B on the train leg, the search3 leg
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gp_gpu.py tests/test_optimizer_gpu.py tests/test_optimizer_parity_gpu.py \
    tests/test_gp_fit_gpu.py tests/test_train_gpu.py tests/test_trajectories_gpu.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/tests_e.log 2>&1 && tail -3 gpurun_out/tests_e.log && \
timeout -k 10 300 python -u scripts/propose_probe.py > gpurun_out/propose_probe_e.log 2>&1 && cat gpurun_out/propose_probe_e.log && \
timeout -k 10 300 python -u scripts/refit_probe.py --n 64 128 256 512 > gpurun_out/refit_probe_e.log 2>&1 && cat gpurun_out/refit_probe_e.log && \
MPO_XCD_SWIZZLE=0 timeout -k 10 300 python -u bench.py --workload train --no-pmc --no-cpu-baseline > gpurun_out/train_xcd0_e.json 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --no-pmc --no-cpu-baseline > gpurun_out/train_xcd1_e.json 2>&1 && \
python -c "
import json
for f in ('gpurun_out/train_xcd0_e.json','gpurun_out/train_xcd1_e.json'):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'])" && \
timeout -k 10 600 python -u bench.py --workload search3 --no-pmc --no-cpu-baseline > gpurun_out/bench_search3_e.json 2> gpurun_out/bench_search3_e.err && cat gpurun_out/bench_search3_e.json
