#!/bin/bash
# Kernel trace of the cl_min chains (configs[3]'s layout at 16 blocks): how much of
# the chains' wall time the GPU spends executing their kernels.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$ROOT/gpurun_out/prof_chain_$TAG"
rm -rf /tmp/prof_chain_$TAG
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats -d /tmp/prof_chain_$TAG -o run --output-format csv \
    -- python "$ROOT/scripts/search_run.py" "$ROOT/gpurun_out/chainprof_$TAG.json" --world-size 33 --block-size 2 \
    --n-fold 5 --num-iterations ${ITERS:-48} --epochs 1 --chain-workers ${WORKERS:-4} \
    > "$ROOT/gpurun_out/chainprof_$TAG.log" 2>&1 && \
find /tmp/prof_chain_$TAG -name "*kernel_stats.csv" -exec cp {} "$ROOT/gpurun_out/prof_chain_$TAG/" \; && \
find /tmp/prof_chain_$TAG -name "*kernel_trace.csv" -exec sh -c 'python3 - "$1" "$2" <<PY
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
ks = collections.Counter(); busy = 0; t0 = None; t1 = 0; spans = []
TRAIN = ("conv_", "conv1_", "pool_", "dense_", "softmax", "adam", "wgrad_reduce", "flip_w2", "colsum", "kfold")
for r in rows:
    name = r["Kernel_Name"]
    if "anonymous namespace" not in name or any(t in name for t in TRAIN):
        continue                      # the GP / acquisition kernels of the refits only
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    spans.append((s, e)); ks[name.split("(")[0][-60:]] += 1
spans.sort()
# union of kernel intervals (time the GPU had at least one kernel running) and the sum
union = 0; cur_s, cur_e = None, None; tot = 0
for s, e in spans:
    tot += e - s
    if cur_e is None or s > cur_e:
        if cur_e is not None: union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None: union += cur_e - cur_s
span = spans[-1][1] - spans[0][0]
with open(sys.argv[2], "w") as fh:
    fh.write(f"GP kernels {len(spans)}  span {span/1e9:.2f} s  union busy {union/1e9:.2f} s  sum {tot/1e9:.2f} s\n")
    for k, c in ks.most_common(25): fh.write(f"{c:8d} {k}\n")
PY' _ {} "$ROOT/gpurun_out/prof_chain_$TAG/trace_summary.txt" \; && \
cat "$ROOT/gpurun_out/prof_chain_$TAG/trace_summary.txt" && ls "$ROOT/gpurun_out/prof_chain_$TAG"
