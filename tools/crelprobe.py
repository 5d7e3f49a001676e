"""Config-5 sweep of the crel gather (csrc/rowtail.hip k_gather_crel): per-call device time of the
inline gather (regcn_layer_rowtail_f32(gather), HIP events after each library call) and the
predict, for several REGCN_CREL_MIN_ITEMS thresholds (0 = every tile gathers its relation rows
per item).  The crel kernel's source rows in flight per wave come from REGCN_CREL_EB (read once
per process).

  python tools/crelprobe.py [--mins 0,512,1024,2048] [--reps 4]
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "re-gcn_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from regcn_amd import _lib  # noqa: E402
from regcn_amd import hyperbolic_layers as HL  # noqa: E402
from regcn_amd.synthetic import CONFIGS, snapshot_series  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mins", default="0,512,1024,2048")
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    cfg = CONFIGS["synthetic_1m"]
    dev = torch.device("cuda", 0)
    snaps = snapshot_series(100, cfg["V"], cfg["R"], cfg["T"] + 1, cfg["per_snap"])
    glist = [bench.prepare_snapshot(cfg["V"], cfg["R"], s, dev) for s in snaps[:cfg["T"]]]
    test = torch.from_numpy(snaps[cfg["T"]][:512]).to(dev)
    del snaps
    model = bench.build_model(cfg, 200, dev, seed=1234)
    model.param_caches = model.memo_pristine = False
    model.use_phases = False  # config 5 runs per-layer launches (bench.py)
    out = {"crel_eb": os.environ.get("REGCN_CREL_EB", "32")}
    for m in [int(v) for v in a.mins.split(",")]:
        HL.CREL_MIN_ITEMS = m
        for g in glist:
            g.__dict__.pop("_crel_tiles", None)
        with torch.no_grad():
            model.predict(glist, cfg["R"], None, test, True)
            torch.cuda.synchronize()
            trace = []
            _lib.EVENT_TRACE = trace
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for _ in range(a.reps):
                _lib.trace_mark("__step__")
                model.predict(glist, cfg["R"], None, test, True)
            s1.record()
            _lib.EVENT_TRACE = None
            torch.cuda.synchronize()
        calls = bench.summarize_trace(trace, a.reps)
        ga = calls.get("regcn_layer_rowtail_f32(gather)", {}).get("ms")
        out[str(m)] = {"gather_ms": round(ga, 4) if ga else None, "predict_ms": round(s0.elapsed_time(s1) / a.reps, 3),
                       "crel_tiles": [g.__dict__.get("_crel_tiles", (0, 0))[1] for g in glist]}
        print(m, out[str(m)], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
