"""Derived per-kernel figures from a pmc_summary.py listing and a rocprofv3 kernel-stats CSV of
the same command: the clock the chip held (GRBM_GUI_ACTIVE / 8 XCDs / mean duration), the MFMA
pipe's busy share (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x those cycles), the L1 <- L2
request stream (TCP_TCC_READ_REQ_sum x 128 B) and the fabric bytes (FETCH_SIZE x 2 + WRITE_SIZE,
in KB; the gfx950 correction of MI355X_MICROARCH.md).

  python tools/pmc_derive.py profiles/r5_c5_pmc_summary.txt profiles/r5_bench_c5_kernel_stats.csv
"""
import csv
import sys


def main():
    summ, stats = sys.argv[1], sys.argv[2]
    pmc, cur = {}, None
    for line in open(summ):
        if not line.startswith(" "):
            cur = line.strip()
            pmc[cur] = {}
        elif cur:
            k, v = line.split()
            pmc[cur][k] = float(v)
    dur = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(stats))}
    print("%-34s %9s %7s %7s %10s %9s %9s" % ("kernel", "us", "GHz", "MFMA%", "L1<-L2 req", "req TB/s", "fabric GB"))
    for k, c in pmc.items():
        name = next((n for n in dur if n.startswith(k[:60])), None)
        if name is None:
            continue
        us = dur[name] / 1e3
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
        ghz = cyc / (us * 1e3) if us else 0
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * cyc) if cyc else 0
        req = c.get("TCP_TCC_READ_REQ_sum", 0)
        fab = (2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / 1e9
        short = k.split("(")[0].replace("void ", "").replace("regcn::", "")
        print("%-34s %9.1f %7.2f %7.1f %10.3g %9.2f %9.2f" % (short[:34], us, ghz, 100 * mfma, req,
                                                            req * 128 / (us * 1e-6) / 1e12, fab))


if __name__ == "__main__":
    main()
