#!/bin/bash
# round 3: where the scatter conv2 input gradient spends its time (MPO_POP_DEBUG=1 skips the MFMA loops)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r}
for D in 0 1; do
( cd /tmp && MPO_POP_DEBUG=$D MPO_DG_SCATTER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T}_$D -o run --output-format csv -- python $GRAFT_REPO_ROOT/scripts/train_probe.py --steps 2 > /tmp/prof_${T}_$D.log 2>&1 ) || exit 1
mkdir -p gpurun_out/prof_dgs_${T}_$D && find /tmp/prof_${T}_$D -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_dgs_${T}_$D/ \;
done
ls gpurun_out/prof_dgs_${T}_0 gpurun_out/prof_dgs_${T}_1
