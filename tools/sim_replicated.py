"""What the owner-partition simulation's replicated time is made of: a rocprofv3 kernel trace of
tools/simprobe.py run with REGCN_SIM_MARKERS=1 (a 1-cycle spin kernel before and after every
simulated rank's launches) is cut at the long blocker spins into steps; in the last `--steps`
steps every kernel outside the marker pairs is work no rank bracket holds (the replicated work,
plus the simulated halo delivery), listed by name with its time per step, beside the wall time
outside the brackets (kernels + gaps).

  python tools/sim_replicated.py gpurun_out/<trace dir>/<name>_results.db [--steps 3]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker-us", type=float, default=50.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = [(int(s), int(e), n) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    spin = [i for i, (s, e, n) in enumerate(rows) if "spin_kernel" in n]
    blockers = [i for i in spin if (rows[i][1] - rows[i][0]) / 1e3 > a.marker_us]
    starts = blockers[-a.steps:]
    ends = starts[1:] + [len(rows)]
    outside = defaultdict(lambda: [0, 0.0])
    wall_out = 0.0
    for b0, b1 in zip(starts, ends):
        inside = False
        last = rows[b0][1]  # the step starts when the blocker ends
        for i in range(b0 + 1, b1):
            s, e, n = rows[i]
            if "spin_kernel" in n and (e - s) / 1e3 <= a.marker_us:
                if not inside:
                    wall_out += max(0, s - last)
                inside = not inside
                last = e
                continue
            if not inside:
                outside[n][0] += 1
                outside[n][1] += (e - s) / 1e3
        if not inside and b1 - 1 > b0:
            wall_out += max(0, rows[b1 - 1][1] - last)
    k = len(starts)
    tot = sum(v[1] for v in outside.values()) / k
    print("steps %d; outside the rank brackets per step: wall %.3f ms, kernels %.3f ms" % (k, wall_out / 1e6 / k, tot / 1e3))
    print("%-100s %8s %10s" % ("kernel", "calls/st", "us/step"))
    for n, (c, t) in sorted(outside.items(), key=lambda kv: -kv[1][1]):
        print("%-100s %8.1f %10.1f" % (n[:100], c / k, t / k))


if __name__ == "__main__":
    main()
