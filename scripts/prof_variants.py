"""rocprofv3 --kernel-trace --stats of the population train step, one run per plan
variant (MPO_POP_PLAN), each kernel_stats.csv copied to gpurun_out/<tag>_<i>.csv
and summarised per kernel family (ms per train step).

  python scripts/prof_variants.py TAG "dgband=0" "dgband=1" [--shard 0/8]
"""
import csv
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    args = sys.argv[2:]
    extra = []
    script = "plan_ab.py"
    if "--dn" in args:            # DenseNet population (scripts/dn_ab.py, MPO_DN_PLAN variants)
        args.remove("--dn")
        script = "dn_ab.py"
    for flag in ("--shard", "--trials", "--members"):
        if flag in args:
            i = args.index(flag)
            extra += [flag, args[i + 1]]
            args = args[:i] + args[i + 2:]
    steps = 3
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    for i, v in enumerate(args):
        d = tempfile.mkdtemp(prefix="mpo_pv_", dir="/tmp")
        cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.join(ROOT, "scripts", script), "--variants", v, "--rounds", "1",
               "--steps", str(steps), *extra]
        r = subprocess.run(cmd, cwd="/tmp", env={**os.environ, "TMPDIR": "/tmp"}, stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, timeout=300)
        if r.returncode != 0:
            print(r.stdout.decode(errors="replace")[-2000:])
            sys.exit(r.returncode)
        paths = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        dst = os.path.join(out_dir, f"{tag}_{i}.csv")
        shutil.copy(paths[0], dst)
        shutil.rmtree(d, ignore_errors=True)
        rows = list(csv.DictReader(open(dst)))
        fam = {}
        for row in rows:
            m = re.search(r"::(\w+)(<[^>]*>)?\(", row["Name"])
            name = m.group(1) if m else row["Name"][:40]
            fam[name] = fam.get(name, 0.0) + float(row["TotalDurationNs"])
        # plan_ab runs 2 warm-up + rounds*steps train steps per variant
        per = 2 + steps
        tot = sum(v_ for k_, v_ in fam.items() if not k_.startswith("__amd"))
        print(f"== {v}: {tot / 1e6 / per:.2f} ms/step of kernel time")
        for k_, v_ in sorted(fam.items(), key=lambda kv: -kv[1])[:14]:
            print(f"   {k_:34s} {v_ / 1e6 / per:8.3f} ms/step")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
