#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, each under its own kill
# timeout) over the EI probe and the training probe; summaries -> gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
pass() {   # tag, counters, program...
  local tag=$1 ctr=$2; shift 2
  ( cd /tmp && timeout -s KILL ${PMC_TIMEOUT:-120} rocprofv3 --pmc $ctr -d "$R/gpurun_out/pmc_$tag" -o pmc \
      --output-format csv -- "$@" > "$R/gpurun_out/pmc_$tag.log" 2>&1 ) && \
  python "$R/scripts/pmc_summary.py" "$R/gpurun_out/pmc_$tag" > "$R/gpurun_out/pmc_$tag.txt" && echo "PMC $tag OK"
}
EI="python $R/scripts/ei_probe.py 3"
TR="python $R/scripts/train_probe.py --steps 1"
pass ei_fetch FETCH_SIZE $EI && pass ei_write WRITE_SIZE $EI && pass ei_sq "$SQ" $EI && \
pass tr_fetch FETCH_SIZE $TR && pass tr_write WRITE_SIZE $TR && pass tr_sq "$SQ" $TR
