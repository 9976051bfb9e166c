#!/bin/bash
# PMC passes over the EI scoring probe for one kernel variant (MPO_GP_KERNEL=wave|block)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-wave}
P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
run() {
  ( cd /tmp && MPO_GP_KERNEL=$V timeout -s KILL 60 rocprofv3 --pmc $2 -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_ei_${V}_$1" -o pmc \
      --output-format csv -- python $GRAFT_REPO_ROOT/scripts/ei_probe.py 3 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_ei_${V}_$1.log" 2>&1 ) \
  && echo "PMC $1 OK" && python scripts/pmc_dump.py gpurun_out/pmc_ei_${V}_$1
}
run p1 "$P1" && run p2 "$P2"
