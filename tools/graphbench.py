"""Snapshot construction benchmark: the device build
(csrc/graphbuild.hip via graph.build_sub_graph_device) next to the host numpy build
(graph.SnapshotGraph, the CPU path) on the BASELINE.json snapshot shapes.

The device build starts from triples already resident in HBM and ends with every list on
the device (the two host reads of the counts included: they are part of a build).  One
JSON line per config on stdout.

  python tools/graphbench.py [--configs icews14s,config5] [--reps 5] [--no-host]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))

from regcn_amd import graph as G  # noqa: E402
from regcn_amd.synthetic import zipf_triples  # noqa: E402

SHAPES = {
    "icews14s": (7128, 230, 246),
    "icews18": (23033, 256, 1540),
    "gdelt": (7691, 240, 770),
    "config5": (1_000_000, 256, 25_000_000),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="icews14s,icews18,gdelt,config5")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-host", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name in a.configs.split(","):
        V, R, T = SHAPES[name]
        rng = np.random.default_rng(0)
        tr = zipf_triples(rng, V, R, T)
        tr_dev = torch.from_numpy(tr).to(dev)
        for _ in range(2):
            G.build_sub_graph_device(V, R, tr_dev, dev)
        torch.cuda.synchronize()
        times = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            g = G.build_sub_graph_device(V, R, tr_dev, dev)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        t_dev = float(np.median(times))
        E = 2 * T
        out = {"config": name, "V": V, "R": R, "triples": T, "edges": E, "device_ms": round(t_dev * 1e3, 3),
               "device_M_edges_per_s": round(E / t_dev / 1e6, 2), "n_tiles": g.n_pos_tiles, "n_heavy": g.n_heavy}
        if not a.no_host:
            t0 = time.perf_counter()
            G.build_sub_graph(V, R, tr, False, 0)
            t_host = time.perf_counter() - t0
            out.update(host_ms=round(t_host * 1e3, 1), host_M_edges_per_s=round(E / t_host / 1e6, 3),
                       host_cores=1, speedup=round(t_host / t_dev, 1))
        print(json.dumps(out), flush=True)
        del g, tr_dev
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
