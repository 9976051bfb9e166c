#!/bin/bash
# round 3: SQ stall breakdown of the training conv kernels (one --pmc pass, 8 SQ counters)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ah}
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES -d $GRAFT_REPO_ROOT/gpurun_out/sq_${T} -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/train_probe.py --steps 1 > $GRAFT_REPO_ROOT/gpurun_out/sq_${T}.log 2>&1 && \
cd $GRAFT_REPO_ROOT && python3 scripts/pmc_dump.py gpurun_out/sq_${T} > gpurun_out/sq_${T}_summary.txt && cat gpurun_out/sq_${T}_summary.txt
