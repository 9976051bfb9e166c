#!/bin/bash
# round 3: scatter conv2 input gradient -- tests, train-step A/B over the LDS budget knob, rocprof of the default
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-u}
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k scatter > gpurun_out/tests_${T}.log 2>&1 && \
  tail -3 gpurun_out/tests_${T}.log && \
MPO_DG_SCATTER=0 timeout -k 10 300 python -u scripts/train_probe.py --steps 6 > gpurun_out/train_gather_${T}.log 2>&1 && grep "train step" gpurun_out/train_gather_${T}.log && \
MPO_DG_SCATTER=1 timeout -k 10 300 python -u scripts/train_probe.py --steps 6 > gpurun_out/train_scatter_${T}.log 2>&1 && grep "train step" gpurun_out/train_scatter_${T}.log && \
MPO_DG_SCATTER=2 timeout -k 10 300 python -u scripts/train_probe.py --steps 6 > gpurun_out/train_hybrid_${T}.log 2>&1 && grep "train step" gpurun_out/train_hybrid_${T}.log && \
MPO_DG_SCATTER=2 MPO_DGS_KB=78 timeout -k 10 300 python -u scripts/train_probe.py --steps 6 > gpurun_out/train_scatter52_${T}.log 2>&1 && grep "train step" gpurun_out/train_scatter52_${T}.log && \
( cd /tmp && MPO_DG_SCATTER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/train_probe.py --steps 4 > /tmp/prof_${T}.log 2>&1 ) && \
mkdir -p gpurun_out/prof_train_scatter_${T} && find /tmp/prof_${T} -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_train_scatter_${T}/ \; && \
( cd /tmp && MPO_DG_SCATTER=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/profg_${T} -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/train_probe.py --steps 4 > /tmp/profg_${T}.log 2>&1 ) && \
mkdir -p gpurun_out/prof_train_gather_${T} && find /tmp/profg_${T} -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_train_gather_${T}/ \; && ls gpurun_out/prof_train_gather_${T}
