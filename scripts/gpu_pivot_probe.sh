cd /tmp
for st in 0 21 22 23; do
  MPO_FIT_DEBUG=$st MPO_FIT_KERNEL=split timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/fp$st -o fit --output-format csv -- python "$GRAFT_REPO_ROOT/scripts/fit_probe.py" --n 500 --kernels split --reps 0 > /tmp/pv$st.log 2>&1 || { grep -v "^[EW]2026" /tmp/pv$st.log | tail -8; exit 1; }
  echo "stop=$st $(grep sw_pivot $(find /tmp/fp$st -name '*kernel_stats.csv') | cut -d, -f4)"
done
