#!/bin/bash
# round 3: blocked 16x16 pivot inverse (MPO_FIT_PIV=blk) -- sklearn-tolerance GP fit tests under it, the sweep share,
# refit probe pair vs blk
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-aa}
MPO_FIT_PIV=blk timeout -k 10 400 python -u -m pytest tests/test_gp_fit_gpu.py tests/test_optimizer_parity_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "sklearn or batching or failure or skopt_oracle" > gpurun_out/tests_${T}.log 2>&1 && \
  tail -3 gpurun_out/tests_${T}.log && \
timeout -k 10 300 python -u scripts/sweep_share_probe.py > gpurun_out/sweep_share_${T}.log 2>&1 && cat gpurun_out/sweep_share_${T}.log && \
MPO_FIT_PIV=blk timeout -k 10 300 python -u scripts/sweep_share_probe.py > gpurun_out/sweep_share_blk_${T}.log 2>&1 && cat gpurun_out/sweep_share_blk_${T}.log && \
MPO_FIT_PIV=pair timeout -k 10 300 python -u scripts/refit_probe.py --n 64 128 256 512 > gpurun_out/refit_probe_pair_${T}.log 2>&1 && cat gpurun_out/refit_probe_pair_${T}.log && \
MPO_FIT_PIV=blk timeout -k 10 300 python -u scripts/refit_probe.py --n 64 128 256 512 > gpurun_out/refit_probe_blk_${T}.log 2>&1 && cat gpurun_out/refit_probe_blk_${T}.log
