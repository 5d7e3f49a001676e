"""Does the CPU oracle track the reference's own CPU path?  (CPU baseline.)

CONTAINER ONLY (imports the read-only reference at /root/reference through the test-only
DGL stand-in of tools/goldens/standin; nothing here runs on the GPU box).  Times, on the
same host cores and inputs, the reference's layer / scorer forward and the oracle
restatement bench.py's `cpu_baseline` leg runs, at the sizes SURVEY.md §8(d) quotes for
the reference (Union V=100k E=1M, Lorentz V=20k E=200k, scorer B=476 N=7,128; d=200),
checks that the two agree numerically, and prints one JSON line per case:

  PYTHONDONTWRITEBYTECODE=1 python tools/cpu_tracking.py [--threads 8] > profiles/r1_cpu_tracking.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "goldens", "standin"))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, REPO)

import torch.nn.functional as F  # noqa: E402
from hyperbolic_src import hyperbolic_decoder as hdec  # noqa: E402
from hyperbolic_src.hyperbolic_layers import HyperbolicUnionRGCNLayer, LorentzRGCNLayer  # noqa: E402
from rgcn import utils as rutils  # noqa: E402

from oracle import graph as og  # noqa: E402
from oracle import layers as ol  # noqa: E402
from oracle import model as om  # noqa: E402

C = 0.01


def triples(seed, V, R, T):
    sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
    from regcn_amd.synthetic import zipf_triples
    return zipf_triples(np.random.default_rng(seed), V, R, T)


def ball(gen, n, d):
    x = torch.randn(n, d, generator=gen)
    x = x / x.norm(dim=1, keepdim=True) * (torch.rand(n, 1, generator=gen) * 2.5 + 0.5) * 0.1
    return x


def timed(fn, reps):
    fn()  # warm (allocator, thread pool)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        t.append(time.perf_counter() - t0)
    return float(np.median(t)), out


def rel_err(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / max(1.0, float(b.abs().max())))


def layer_case(kind, V, R, T, d, reps):
    tr = triples(7, V, R, T)
    gen = torch.Generator().manual_seed(7)
    h = ball(gen, V, d)
    rel = torch.randn(2 * R, d, generator=gen) * 0.3
    torch.manual_seed(7)
    if kind == "union":
        lay = HyperbolicUnionRGCNLayer(d, d, 2 * R, -1, c=C, activation=F.rrelu, self_loop=True,
                                       radius_msg_gamma=0.15).eval()
    else:
        lay = LorentzRGCNLayer(d, d, 2 * R, 100, c=C, activation=F.rrelu, self_loop=True).eval()
    rg = rutils.build_sub_graph(V, R, tr, False, "cpu")
    g = og.build_sub_graph(V, R, tr)
    E = int(rg.number_of_edges())
    with torch.no_grad():
        t_ref, y_ref = timed(lambda: lay(rg, h, rel), reps)
        sd = {k: v for k, v in lay.state_dict().items()}
        if kind == "union":
            t_or, y_or = timed(lambda: ol.union_layer(g, h, rel, sd["weight_neighbor"], sd["loop_weight"],
                                                      sd["evolve_loop_weight"], C, 0.15), reps)
        else:
            t_or, y_or = timed(lambda: ol.lorentz_layer(g, h, rel, sd["weight"], sd["loop_weight"],
                                                        sd["evolve_loop_weight"], C, 100), reps)
    return {"case": kind + "_layer", "V": V, "E": E, "d": d, "reference_s": round(t_ref, 3),
            "oracle_s": round(t_or, 3), "reference_M_edges_per_s": round(E / t_ref / 1e6, 4),
            "oracle_M_edges_per_s": round(E / t_or / 1e6, 4), "oracle_over_reference_time": round(t_or / t_ref, 3),
            "max_rel_err": rel_err(y_or, y_ref)}


def score_case(B, N, d, reps):
    gen = torch.Generator().manual_seed(9)
    q, e = ball(gen, B, d) * 10, ball(gen, N, d) * 10
    bias = torch.randn(N, generator=gen) * 0.1
    with torch.no_grad():
        t_ref, s_ref = timed(lambda: hdec._chunked_hyperbolic_dist_score(q, e, bias, C, 128, 2048), reps)
        t_or, s_or = timed(lambda: om.dist_score(q, e, bias, C), reps)
    return {"case": "score", "B": B, "N": N, "d": d, "reference_s": round(t_ref, 3), "oracle_s": round(t_or, 3),
            "reference_M_pairs_per_s": round(B * N / t_ref / 1e6, 3), "oracle_M_pairs_per_s": round(B * N / t_or / 1e6, 3),
            "oracle_over_reference_time": round(t_or / t_ref, 3), "max_rel_err": rel_err(s_or, s_ref)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cases", default="union,lorentz,score")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    for case in a.cases.split(","):
        if case == "union":
            r = layer_case("union", 100_000, 256, 500_000, 200, a.reps)
        elif case == "lorentz":
            r = layer_case("lorentz", 20_000, 256, 100_000, 200, a.reps)
        else:
            r = score_case(476, 7128, 200, a.reps)
        r["threads"] = a.threads
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
