"""Config 5 with independent predicts in flight on separate streams: the bench's two windows
(|V| = 1M, |E| = 50M per snapshot, history 3), K predicts alternating between them, issued on 1 or
2 (or more) streams; wall time per predict over the same K.  Does the MFMA-bound tail of one
predict overlap the L2-bound gathers of another?

  python tools/c5_concurrency.py [--steps 12] [--streams 1,2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--streams", default="1,2")
    a = ap.parse_args()
    from regcn_amd.synthetic import CONFIGS, snapshot_series
    cfg = CONFIGS["synthetic_1m"]
    dev = torch.device("cuda", 0)
    V, R, T = cfg["V"], cfg["R"], cfg["T"]
    snaps = snapshot_series(100, V, R, T + 2, cfg["per_snap"])
    graphs = [bench.prepare_snapshot(V, R, s, dev) for s in snaps[:T + 1]]
    tests = [torch.from_numpy(np.ascontiguousarray(snaps[T + i][:512])).to(dev) for i in range(2)]
    del snaps
    windows = [graphs[i:i + T] for i in range(2)]
    model = bench.build_model(cfg, 200, dev, seed=1234)
    model.use_phases = False
    model.memo_pristine = model.param_caches = False
    with torch.no_grad():
        ref = [model.predict(windows[k], R, None, tests[k], True)[1].clone() for k in range(2)]
    torch.cuda.synchronize()
    for ns in (int(x) for x in a.streams.replace("+", ",").split(",")):
        streams = [torch.cuda.Stream(dev) for _ in range(ns)]
        cur = torch.cuda.current_stream(dev)
        with torch.no_grad():
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for st in streams:
                    st.wait_stream(cur)
                outs = []
                for k in range(a.steps):
                    with torch.cuda.stream(streams[k % ns]):
                        outs.append(model.predict(windows[k % 2], R, None, tests[k % 2], True)[1])
                for st in streams:
                    cur.wait_stream(st)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 1e3 / a.steps
                same = all(torch.equal(o, ref[k % 2]) for k, o in enumerate(outs))
                del outs
        print(json.dumps({"streams": ns, "ms_per_predict": round(ms, 3), "scores_bitwise_equal": same,
                          "M_edges_per_s": round(3e8 / ms / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
