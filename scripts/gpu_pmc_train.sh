#!/bin/bash
# Detailed PMC passes over the training probe (one counter group per run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
PROG="python $R/scripts/train_probe.py --steps 1 ${PROBE_ARGS}"
pass() {
  local tag=$1 ctr=$2
  ( cd /tmp && rm -rf /tmp/pmc_$tag && timeout -s KILL ${PMC_TIMEOUT:-150} rocprofv3 --pmc $ctr -d /tmp/pmc_$tag -o pmc \
      --output-format csv -- $PROG > "$R/gpurun_out/pmc_$tag.log" 2>&1 ) && \
  python "$R/scripts/pmc_dump.py" /tmp/pmc_$tag > "$R/gpurun_out/pmc_$tag.txt" && echo "PMC $tag OK"
}
pass A "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" && \
pass B "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_WAVES GRBM_GUI_ACTIVE" && \
pass C "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
