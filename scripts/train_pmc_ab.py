"""HBM bytes per train batch by kernel family for plan variants (MPO_POP_PLAN),
measured as bench.py measures them (separate FETCH_SIZE / WRITE_SIZE rocprofv3
passes over scripts/train_probe.py --no-eval, FETCH_SIZE doubled).

  python scripts/train_pmc_ab.py "xcd=0" "xcd=1"
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    prog = [os.path.join(bench.ROOT, "scripts", "train_probe.py"), "--steps", "1", "--no-eval"]
    ours = lambda k: "anonymous namespace" in k   # noqa: E731
    out = {}
    for v in sys.argv[1:]:
        os.environ["MPO_POP_PLAN"] = v
        rf, rw = bench.pmc_pass(["FETCH_SIZE"], prog), bench.pmc_pass(["WRITE_SIZE"], prog)
        fam = bench._per_kernel_bytes(rf, rw, ours, 3, family=True)
        busy, per = bench.mfma_busy(bench.pmc_pass(["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"], prog),
                                    bench.PMC_FAMILIES)
        out[v] = {"total_GB": sum(fam.values()) / 1e9, "mfma_busy": busy, "per_family_mfma_busy": per,
                  "per_family_GB": {k: round(b / 1e9, 3) for k, b in fam.items()}}
        print(v, json.dumps(out[v]), flush=True)


if __name__ == "__main__":
    main()
