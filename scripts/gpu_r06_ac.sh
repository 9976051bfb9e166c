#!/bin/bash
# r06 session ac: which change segfaults the lone-chain probe (Python faulthandler)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "MPO_FIT_GRAPH=0 MPO_FIT_POOLED=0" "MPO_FIT_GRAPH=1 MPO_FIT_POOLED=0" "MPO_FIT_GRAPH=0 MPO_FIT_POOLED=1"; do
  echo "== $v" >> gpurun_out/ac_chain.log
  env $v timeout -k 10 120 python -X faulthandler -u scripts/ask_chain_probe.py --ask-n 2 --reps 1 >> gpurun_out/ac_chain.log 2>&1
  echo "rc=$?" >> gpurun_out/ac_chain.log
done
