#!/bin/bash
# r06 session bg: DenseNet third weight-gradient stream re-measured with the BN reduce fusion on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/dn_ab.py --variants "wgs=2" "wgs=3" "wgs=2" "wgs=3" "wgs=2" "wgs=3" --rounds 4 --steps 5 > gpurun_out/bg_ab.log 2>&1
