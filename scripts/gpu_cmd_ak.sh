#!/bin/bash
# round 3: LML launch sequence at small n -- kernel durations vs the per-launch time (gaps between the kernels)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-ak}
for N in 64 128; do
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/prof_${T}_$N -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/refit_probe.py --n $N > $GRAFT_REPO_ROOT/gpurun_out/prof_${T}_$N.log 2>&1 ) || exit 1
  mkdir -p gpurun_out/prof_${T}_$N && find /tmp/prof_${T}_$N -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_${T}_$N/ \;
  cat gpurun_out/prof_${T}_$N.log | grep 'n='
  python3 - <<PY
import csv
rows=list(csv.DictReader(open("gpurun_out/prof_${T}_$N/run_kernel_stats.csv")))
for r in rows[:12]:
    print("%6.2f%% %6d calls %8.2f us  %s"%(float(r['Percentage']),int(r['Calls']),float(r['AverageNs'])/1e3,r['Name'][:90]))
PY
done
