"""Per-step kernel breakdown of a rocprofv3 kernel trace (rocpd sqlite) over the timed region of
tools/simprobe.py / bench.py: the dispatches from the `--from`-th launch of the marker kernel
(default: the initial-state kernel, one per step; the first is the warm-up step) to the end.

  python tools/simprof_summary.py <results.db> [--marker k_init_rows4<11>] [--from 1] [--steps 3]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="k_init_rows4<11>")
    ap.add_argument("--from", dest="start", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(idx) <= a.start:
        raise SystemExit("marker %r seen %d times" % (a.marker, len(idx)))
    tail = rows[idx[a.start]:]
    span = (tail[-1][2] - tail[0][1]) / 1e6
    agg = {}
    for n, s, e, gx, wx in tail:
        v = agg.setdefault(n, [0, 0, gx // max(wx, 1)])
        v[0] += 1
        v[1] += e - s
    busy = sum(v[1] for v in agg.values())
    print("dispatches %d, markers at %s; timed span %.3f ms = %.3f ms per step; kernel busy %.3f ms per step"
          % (len(rows), idx, span, span / a.steps, busy / 1e6 / a.steps))
    print("%-90s %8s %10s %10s %8s" % ("kernel", "calls/st", "ms/step", "us/call", "wgs"))
    for n, (k, t, wg) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print("%-90s %8.1f %10.3f %10.1f %8d" % (n[:90], k / a.steps, t / 1e6 / a.steps, t / k / 1e3, wg))


if __name__ == "__main__":
    main()
