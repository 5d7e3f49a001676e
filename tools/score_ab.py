"""A/B of scorer variants: tools/scorebench.py (score mode, HIP-event time per launch) under
each environment setting of --var (default REGCN_SCORE32 = 0 / 1: the v_mfma_f32_16x16x4f32 and
v_mfma_f32_32x32x2f32 kernels), alternated, at config 5 (B = 1024, N = 1M) and the ICEWS14s
decoder shape (B = 492, N = 7128).

  python tools/score_ab.py [--rounds 2] [--var REGCN_SCORE_NT]
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--var", default="REGCN_SCORE32")
    ap.add_argument("--shapes", default="1024x1000000,492x7128",
                    help="B x N pairs, comma- or plus-separated (ICEWS18: 3080x23033, GDELT: 1540x7691)")
    a = ap.parse_args()
    for shp in a.shapes.replace("+", ",").split(","):
        B, N = (int(v) for v in shp.split("x"))
        reps = 5 if N >= 100_000 else 200
        for rnd in range(a.rounds):
            for v in ("0", "1"):
                env = dict(os.environ, **{a.var: v})
                r = subprocess.run([sys.executable, os.path.join(HERE, "scorebench.py"), "--B", str(B), "--N", str(N),
                                    "--modes", "score", "--reps", str(reps)], env=env, capture_output=True, text=True,
                                   timeout=300)
                if r.returncode:
                    print(r.stderr[-2000:], file=sys.stderr)
                    raise SystemExit(r.returncode)
                res = json.loads(r.stdout.strip().splitlines()[-1])
                print(json.dumps({"B": B, "N": N, "round": rnd, a.var: int(v), **res["score"]}), flush=True)


if __name__ == "__main__":
    main()
