#!/bin/bash
# round 3, run k: the configs[3]-layout search leg (GP in the loop) + the refit probe, after the fused / paired LML sweep and the fused EI finish
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-k}
timeout -k 10 900 python -u bench.py --workload search3 --steps 1 --warmup 0 > gpurun_out/search3_${T}.json 2> gpurun_out/search3_${T}.err && cat gpurun_out/search3_${T}.json
