"""Config-5 owner-partition rank simulation alone (bench.owner_simulation), for profiling the
per-rank launches:  python tools/simprobe.py [--world 8] [--chunks 0]"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from regcn_amd.synthetic import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--chunks", type=int, default=0, help="pipeline chunks per rank (0: auto)")
    a = ap.parse_args()
    if a.chunks:
        from regcn_amd import parallel
        parallel.owner_chunks = lambda V, world: a.chunks
    args = argparse.Namespace(d=200, queries=1024)
    cfg = dict(CONFIGS["synthetic_1m"])
    res = bench.owner_simulation(args, cfg, torch.device("cuda", 0), a.world)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
