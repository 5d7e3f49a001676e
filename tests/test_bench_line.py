"""The bench line the driver parses (bench.py compact_line): a recorded full bench record
(profiles/r5_bench_final.json, the 21 KB line round 5's driver could not parse) must come out
as one JSON line under 8 KB that still carries the contract keys, the headline's roofline and
cpu_baseline, the owner simulation and every dataset leg."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _record():
    with open(os.path.join(REPO, "profiles", "r5_bench_final.json")) as fh:
        out = json.load(fh)
    # a configs[0] leg as run_regcn returns it
    out["icews14s_regcn"] = {"value": 5.0, "ms_per_step": 0.6, "latency_ms_per_predict": None,
                             "cpu_baseline": {"value": 0.01, "unit": "M edges/s", "cores": 16, "kind": "port",
                                              "sample": "x"},
                             "mrr_parity": {"entity": {"max_abs_delta": 0.0}, "relation": {"max_abs_delta": 0.0}}}
    return out


def test_compact_line_parses_and_fits():
    import bench
    out = _record()
    assert len(json.dumps(out)) > bench.LINE_LIMIT  # the recorded line itself is too long
    s = bench.compact_line(out, "gpurun_out/bench_detail.json")
    assert "\n" not in s
    assert len(s.encode()) <= bench.LINE_LIMIT
    line = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    assert line["value"] == out["value"] and line["ms_per_step"] == out["ms_per_step"]
    assert "snapshot_stats" not in line["config"]
    rf = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_frac"):
        assert k in rf, k
    assert rf["l2_request_stream"]["achieved_TBps"] > 0
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference")
    sim = line["owner_simulation"]
    assert sim["predicted_step_ms"] > 0 and sim["max_rank_ms"] > 0 and "exposed_exchange_ms" in sim
    for leg in ("icews14s", "icews14s_regcn", "icews18", "gdelt", "gdelt_lgcn"):
        assert line["legs"][leg]["value"] > 0, leg
    assert line["legs"]["icews14s"]["roofline"]["frac"] > 0
    assert line["legs"]["gdelt"]["cpu_baseline"]["value"] > 0
    assert line["legs"]["icews14s_regcn"]["cpu_baseline"]["value"] > 0


def test_compact_line_drops_optional_blocks_before_overflowing():
    import bench
    out = _record()
    out["config"]["workload"] = "w" * 5000  # an oversized field is cut, the line stays parseable
    s = bench.compact_line(out)
    assert len(s.encode()) <= bench.LINE_LIMIT
    assert json.loads(s)["roofline"]["frac"] > 0
