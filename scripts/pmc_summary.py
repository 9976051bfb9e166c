"""Summarise a rocprofv3 --pmc csv per kernel family (diagnostic)."""
import collections
import csv
import glob
import sys

def family(n):
    if "conv_img_kernel<0" in n: return "conv1_fwd"
    if "conv_img_kernel<1" in n: return "conv2_fwd"
    if "conv_dgrad" in n: return "conv2_dgrad"
    if "conv_wgrad_kernel<1" in n: return "conv2_wgrad"
    if "conv_wgrad_kernel<0" in n: return "conv1_wgrad"
    if "gp_score" in n: return "gp_score"
    if "(anonymous namespace)::" in n: return n.split("(anonymous namespace)::")[1].split("(")[0].split("<")[0]
    return None


def main():
    path = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    disp = collections.defaultdict(set)
    for r in rows:
        key = family(r["Kernel_Name"])
        if key is None:
            continue
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(key, r["Counter_Name"])] += 1
        disp[key].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    for key, d in sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        g = d.get("GRBM_GUI_ACTIVE", 0)
        line = "%-16s launches=%d" % (key, len(disp[key]))
        if g:
            line += " gui=%.3gk" % (g / 1e3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and g:
            line += " mfma_util=%.1f%%" % (100 * d["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024))
        if "SQ_WAVE_CYCLES" in d:
            w = d["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in d:
                    line += " %s=%.0f%%" % (c.replace("SQ_", "").lower(), 100 * d[c] / w)
        if "SQ_LDS_IDX_ACTIVE" in d and d["SQ_LDS_IDX_ACTIVE"]:
            line += " lds_conflict=%.1f%%" % (100 * d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_LDS_IDX_ACTIVE"])
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            if c in d:
                line += " %s=%.1fMB (%.3fMB/launch)" % (c, d[c] / 1024, d[c] / 1024 / max(1, len(disp[key])))
        print(line)


if __name__ == "__main__":
    main()
