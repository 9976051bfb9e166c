#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: 2 ranks sharing cuda:0 over gloo
# (RCCL refuses two ranks on one device).  Not a scaling measurement.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for wl in ${WORKLOADS:-ei train search}; do
  # bench.py --gpus 2 without WORLD_SIZE launches torch.distributed.run itself (the driver's SCALE form)
  MPO_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 --workload $wl \
      --train-trials 8 --train-steps 2 --no-cpu-baseline --no-pmc \
      > gpurun_out/rehearse_$wl.json 2> gpurun_out/rehearse_$wl.err || { tail -20 gpurun_out/rehearse_$wl.err; exit 1; }
  echo "$wl: $(head -c 400 gpurun_out/rehearse_$wl.json)"
done
