#!/bin/bash
# round 3: blocked pivot inverse timing A/B (sweep share, refit probe pair vs blk) and the accuracy tests without -x
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ab}
timeout -k 10 300 python -u scripts/sweep_share_probe.py > gpurun_out/sweep_share_${T}.log 2>&1 && cat gpurun_out/sweep_share_${T}.log && \
MPO_FIT_PIV=blk timeout -k 10 300 python -u scripts/sweep_share_probe.py > gpurun_out/sweep_share_blk_${T}.log 2>&1 && cat gpurun_out/sweep_share_blk_${T}.log && \
MPO_FIT_PIV=pair timeout -k 10 300 python -u scripts/refit_probe.py --n 64 128 256 512 > gpurun_out/refit_probe_pair_${T}.log 2>&1 && cat gpurun_out/refit_probe_pair_${T}.log && \
MPO_FIT_PIV=blk timeout -k 10 300 python -u scripts/refit_probe.py --n 64 128 256 512 > gpurun_out/refit_probe_blk_${T}.log 2>&1 && cat gpurun_out/refit_probe_blk_${T}.log || exit $?
MPO_FIT_PIV=blk timeout -k 10 300 python -u -m pytest tests/test_gp_fit_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "sklearn" > gpurun_out/tests_blk_${T}.log 2>&1
rc=$?; tail -12 gpurun_out/tests_blk_${T}.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gp_fit_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "sklearn" > gpurun_out/tests_pair_${T}.log 2>&1
rc=$?; tail -5 gpurun_out/tests_pair_${T}.log; exit $rc
