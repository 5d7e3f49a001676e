"""L1 <- L2 read requests of the config-5 inline gather per library call, from a rocprofv3
`--pmc TCP_TCC_READ_REQ_sum` run of the bench command (one gather call = one k_gather_crel
launch over the big tiles + one k_gather_agg launch over the rest).  Writes the JSON bench.py's
l2_request_stream reads:

  python tools/pmc_l2req.py gpurun_out/<pmc dir> --config synthetic_1m > profiles/pmc_l2req_synthetic_1m.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

GATHER = ("k_gather_crel", "k_gather_agg")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default="synthetic_1m")
    ap.add_argument("--counter", default="TCP_TCC_READ_REQ_sum")
    a = ap.parse_args()
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == a.counter and any(k in r["Kernel_Name"] for k in GATHER):
                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    kernels = {k: {"launches": len(v), "requests_per_launch": sum(v) / len(v)} for k, v in vals.items()}
    total = sum(k["requests_per_launch"] for k in kernels.values())
    print(json.dumps({"config": a.config, "counter": a.counter, "gather_requests_per_launch": total,
                      "kernels": kernels,
                      "note": "one gather call = one launch of each kernel listed; 128 B per request"}, indent=1))


if __name__ == "__main__":
    main()
