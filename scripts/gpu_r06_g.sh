#!/bin/bash
# r06 session g: DenseNet 1x1 weight gradient fed by float4 loads (bits + time + kernel stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/dn_ab.py --variants "wg1v=0" "wg1v=1" --rounds 6 --steps 5 > gpurun_out/g_dn_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/prof_variants.py g --dn "wg1v=0" "wg1v=1" > gpurun_out/g_prof.log 2>&1
