"""Mean per-dispatch PMC values per kernel from rocprofv3 --pmc csv output directories.

  python tools/pmc_summary.py gpurun_out/pmc_l2 gpurun_out/pmc_sq [--match k_rowtail,k_layer]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[r["Kernel_Name"]][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
    return out


def main():
    dirs = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    for a in sys.argv[1:]:
        if a.startswith("--match="):
            match = a.split("=", 1)[1].split(",")
    res = defaultdict(dict)
    for d in dirs:
        for k, cs in load(d).items():
            if match and not any(m in k for m in match):
                continue
            for c, vals in cs.items():
                per = defaultdict(float)
                for did, v in vals:
                    per[did] += v
                res[k][c] = sum(per.values()) / len(per)
    for k, cs in sorted(res.items()):
        print(k[:70])
        for c, v in sorted(cs.items()):
            print("    %-28s %.4g" % (c, v))


if __name__ == "__main__":
    main()
