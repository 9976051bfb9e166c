"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_summary.json,
the file bench.py reads for ``roofline.traffic``.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for streaming stores.

usage: python scripts/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> <key> [launch_div]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(d, counter, needle):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = [float(r["Counter_Value"]) * 1024.0 for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and needle in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no {counter} rows for {needle} in {path}")
    return sum(vals) / len(vals), len(vals)


def main():
    fdir, wdir, needle, key = sys.argv[1:5]
    fetch, nf = per_launch(fdir, "FETCH_SIZE", needle)
    write, nw = per_launch(wdir, "WRITE_SIZE", needle)
    out_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    d.setdefault(needle, {})[key] = {
        "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
        "hbm_bytes_per_launch": 2.0 * fetch + write,
        "launches": [nf, nw],
        "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE as counted",
        "source": "rocprofv3 --pmc passes (scripts/gpu_pmc_all.sh); summaries under profiles/r01/pmc_*",
    }
    json.dump(d, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(d[needle][key]))


if __name__ == "__main__":
    main()
