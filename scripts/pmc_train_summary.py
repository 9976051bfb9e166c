"""Fold the training-probe PMC passes (scripts/gpu_pmc_all.sh: tr_sq, tr_fetch,
tr_write over `train_probe.py --steps 1` = 3 train steps) into
profiles/pmc_summary.json["population_step"], which bench.py reports.

* MFMA busy per kernel family = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
  (the counter adds the issue cycles of every MFMA: 32 per v_mfma_f32_16x16x4_f32);
  the population step's figure is the GUI-time-weighted mean over the MFMA kernels.
* HBM bytes per train step = (2 x FETCH_SIZE + WRITE_SIZE) / 3 over every kernel of the
  probe (FETCH_SIZE doubled as MI355X_MICROARCH.md prescribes for wide streaming reads;
  the gathers of the conv kernels are uncalibrated widths -- an estimate).

usage: python scripts/pmc_train_summary.py <tr_sq dir> <tr_fetch dir> <tr_write dir> [steps]
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import family  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MFMA_FAMILIES = ("conv1_fwd", "conv2_fwd", "conv2_dgrad", "conv2_wgrad", "conv1_wgrad", "dense_kernel")


def rows(d):
    return list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0])))


def main():
    sq, fe, wr = sys.argv[1:4]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows(sq):
        f = family(r["Kernel_Name"])
        if f:
            agg[f][r["Counter_Name"]] += float(r["Counter_Value"])
    per = {}
    num = den = 0.0
    for f in MFMA_FAMILIES:
        g = agg[f].get("GRBM_GUI_ACTIVE", 0.0)
        if not g:
            continue
        busy = agg[f]["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024)
        per[f] = {"mfma_busy": busy, "gui_cycles_per_step": g / 8 / steps,
                  "lds_bank_conflict": agg[f].get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, agg[f].get("SQ_LDS_IDX_ACTIVE", 0.0))}
        num += busy * g
        den += g
    fetch = sum(float(r["Counter_Value"]) for r in rows(fe) if r["Counter_Name"] == "FETCH_SIZE") * 1024
    write = sum(float(r["Counter_Value"]) for r in rows(wr) if r["Counter_Name"] == "WRITE_SIZE") * 1024
    out_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    d["population_step"] = {
        "mfma_busy": num / den, "mfma_busy_kernels": list(per), "per_kernel": per,
        "hbm_bytes_per_train_step": (2 * fetch + write) / steps,
        "fetch_size_bytes_raw_per_train_step": fetch / steps, "write_size_bytes_per_train_step": write / steps,
        "workload": "train_probe.py: 64 trials x 5 folds = 320 members, batch 100",
        "source": "rocprofv3 --pmc passes (scripts/gpu_pmc_all.sh); summaries under profiles/r01/pmc_tr_*",
    }
    json.dump(d, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(d["population_step"], indent=1))


if __name__ == "__main__":
    main()
