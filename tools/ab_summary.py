"""One line per A/B variant: ms per step of the plain run and the average duration of the
headline's main kernels from the rocprofv3 --stats csv of the traced run (tools/lib_ab.sh)."""
import csv
import glob
import json
import os
import sys

KEYS = ["k_rowtail2", "k_rowtail3", "k_gather_agg", "k_gather_crel", "k_union_runs", "k_score_f32_jobs",
        "k_gather_sum", "k_init_rows4"]


def main():
    name, line, prof = sys.argv[1:4]
    ms = None
    for ln in open(line):
        ln = ln.strip()
        if ln.startswith("{"):
            ms = json.loads(ln).get("ms_per_step")
    avg = {}
    for f in glob.glob(os.path.join(prof, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            full = r["Name"].split("(")[0].replace("void ", "").replace("regcn::", "")
            if full.split("<")[0] in KEYS:
                avg[full] = float(r["AverageNs"]) / 1e3
    print(json.dumps({"var": name, "ms_per_step": ms, "us": {k: round(v, 1) for k, v in avg.items()}}), flush=True)


if __name__ == "__main__":
    main()
