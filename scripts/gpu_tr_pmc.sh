#!/bin/bash
# one SQ counter pass over the MNIST training bench leg; per-kernel (with template args) sums
cd /tmp && rm -rf /tmp/tpmc && timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    -d /tmp/tpmc -o pmc --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --workload train --no-cpu-baseline --no-pmc --train-steps 2 > /tmp/tpmc.log 2>&1 || { tail -5 /tmp/tpmc.log; exit 1; }
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out/trpmc" && cp $(find /tmp/tpmc -name "*counter_collection.csv") "$GRAFT_REPO_ROOT/gpurun_out/trpmc/"
python3 - <<'PY'
import csv, glob, os, re, collections
f = glob.glob(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/trpmc/*counter_collection.csv")[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    m = re.search(r"::(\w+(<[^>]*>)?)\(", r["Kernel_Name"])
    if not m: continue
    agg[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"])[:16]:
    g = c["GRBM_GUI_ACTIVE"] or 1
    simd = g * 1024 / 8
    print("%-30s gui %.3g  mfma_busy %.1f%%  lds_conflict %.1f%%  wait_any/wave %.2f  active_any/wave %.2f  waves/simd %.2f" % (
        k, g, 100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd, 100 * c["SQ_LDS_BANK_CONFLICT"] / max(1, c["SQ_LDS_IDX_ACTIVE"]),
        c["SQ_WAIT_INST_ANY"] / max(1, c["SQ_WAVE_CYCLES"]), c["SQ_ACTIVE_INST_ANY"] / max(1, c["SQ_WAVE_CYCLES"]),
        c["SQ_WAVE_CYCLES"] / simd))
PY
