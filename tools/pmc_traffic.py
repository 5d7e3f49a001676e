"""Per-launch HBM traffic of each kernel from rocprofv3 PMC counter collections.

Usage (after two separate counter passes of the same bench command on the GPU box):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py ...
  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --config icews14s_lgcn_roth --d 200 \
      > profiles/pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are reported in KiB.  Per /opt/skills/guides/MI355X_MICROARCH.md
(HBM section), gfx950 FETCH_SIZE counts half the bytes of wide (16 B/lane) streaming
reads, so it is doubled; WRITE_SIZE is exact.  Both count L2 -> fabric requests, i.e.
Infinity-Cache hits are included (an upper bound on true HBM bytes at these sizes).
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def _load(dirname):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % dirname)
    per = collections.defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def short(name):
    m = re.search(r"regcn::(k_[A-Za-z0-9_]+(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--config", required=True)
    ap.add_argument("--d", type=int, default=200)
    a = ap.parse_args()
    fetch, write = _load(a.fetch_dir), _load(a.write_dir)
    out = {}
    for name in sorted(set(fetch) & set(write)):
        if "regcn::" not in name:
            continue
        f_kib = sum(fetch[name]) / len(fetch[name])
        w_kib = sum(write[name]) / len(write[name])
        fb, wb = 2.0 * f_kib * 1024, w_kib * 1024
        out[short(name)] = dict(launches=len(fetch[name]), fetch_size_kib=round(f_kib, 1),
                                write_size_kib=round(w_kib, 1), read_bytes=round(fb), write_bytes=round(wb),
                                hbm_bytes=round(fb + wb))
    print(json.dumps({"config": a.config, "d": a.d, "counters": "FETCH_SIZE x2 (gfx950) + WRITE_SIZE",
                      "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
