#!/bin/bash
# r06 session az: bench train leg, final plan vs the r06 plan before conv_kb1 / wgpair, alternating on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "xcd=4" "conv_kb1=40,wgpair=0" "xcd=4" "conv_kb1=40,wgpair=0"; do
  MPO_POP_PLAN="$v" timeout -k 10 200 python -u bench.py --workload train --no-pmc --no-cpu-baseline > gpurun_out/az_tmp.json 2> gpurun_out/az_tmp.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/az_tmp.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" "$v" >> gpurun_out/az_ab.log
done
