"""A/B of the scorer's MFMA shape: tools/scorebench.py (score mode, HIP-event time per launch)
with REGCN_SCORE32=0 (v_mfma_f32_16x16x4f32 kernel) and =1 (v_mfma_f32_32x32x2f32 kernel),
alternated, at config 5 (B = 1024, N = 1M) and the ICEWS14s decoder shape (B = 492, N = 7128).

  python tools/score_ab.py [--rounds 2]
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
    a = ap.parse_args()
    for B, N, reps in ((1024, 1_000_000, 5), (492, 7128, 200)):
        for rnd in range(a.rounds):
            for v in ("0", "1"):
                env = dict(os.environ, REGCN_SCORE32=v)
                r = subprocess.run([sys.executable, os.path.join(HERE, "scorebench.py"), "--B", str(B), "--N", str(N),
                                    "--modes", "score", "--reps", str(reps)], env=env, capture_output=True, text=True,
                                   timeout=300)
                if r.returncode:
                    print(r.stderr[-2000:], file=sys.stderr)
                    raise SystemExit(r.returncode)
                res = json.loads(r.stdout.strip().splitlines()[-1])
                print(json.dumps({"B": B, "N": N, "round": rnd, "score32": int(v), **res["score"]}), flush=True)


if __name__ == "__main__":
    main()
