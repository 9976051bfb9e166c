#!/bin/bash
# one SQ counter pass over the DenseNet bench leg; per-kernel-family sums
cd /tmp && rm -rf /tmp/dpmc && timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    -d /tmp/dpmc -o pmc --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --workload densenet --no-cpu-baseline --no-pmc --train-steps 2 > /tmp/dpmc.log 2>&1 || { tail -5 /tmp/dpmc.log; exit 1; }
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out/dnpmc" && cp $(find /tmp/dpmc -name "*counter_collection.csv") "$GRAFT_REPO_ROOT/gpurun_out/dnpmc/"
python3 - <<'PY'
import csv, glob, os, re, collections
f = glob.glob(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/dnpmc/*counter_collection.csv")[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    m = re.search(r"::(dn_\w+)", r["Kernel_Name"])
    if not m: continue
    agg[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(agg.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"]):
    g = c["GRBM_GUI_ACTIVE"] or 1
    simd = g * 1024 / 8   # SIMD-cycles (GRBM counts per XCD, 8 XCDs)
    print("%-24s gui %.3g  mfma_busy %.1f%%  lds_conflict %.1f%%  wait_any/wave %.2f  active_any/wave %.2f" % (
        k, g, 100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd, 100 * c["SQ_LDS_BANK_CONFLICT"] / max(1, c["SQ_LDS_IDX_ACTIVE"]),
        c["SQ_WAIT_INST_ANY"] / max(1, c["SQ_WAVE_CYCLES"]), c["SQ_ACTIVE_INST_ANY"] / max(1, c["SQ_WAVE_CYCLES"])))
PY
