#!/bin/bash
# round 3: DenseNet BN-backward sums fused into the input-gradient conv -- DenseNet GPU suites, bench leg A/B, rocprof
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-x}
timeout -k 10 400 python -u -m pytest tests/test_densenet_gpu.py tests/test_trajectories_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "densenet or DenseNet or fused or isolation or trajectory or forward or fit_folds or routes" > gpurun_out/tests_${T}.log 2>&1 && \
  tail -3 gpurun_out/tests_${T}.log && \
MPO_DN_BNFUSE=0 timeout -k 10 300 python -u bench.py --workload densenet --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/dn_unfused_${T}.json 2> gpurun_out/dn_unfused_${T}.err && cat gpurun_out/dn_unfused_${T}.json && \
timeout -k 10 300 python -u bench.py --workload densenet --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/dn_fused_${T}.json 2> gpurun_out/dn_fused_${T}.err && cat gpurun_out/dn_fused_${T}.json && \
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --workload densenet --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > /tmp/prof_${T}.log 2>&1 ) && \
mkdir -p gpurun_out/prof_dn_${T} && find /tmp/prof_${T} -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_dn_${T}/ \; && ls gpurun_out/prof_dn_${T}
