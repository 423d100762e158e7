"""Per-launch efficiency of the binomial step kernel from a rocprofv3 kernel-trace CSV
(tools/profile.sh output): the launches of ONE serialised pass, step r covering positions 1..r of
`cols` table columns (fused pass at n=1024, U=4: 2 n x 4 = 8192 columns of L = 128 positions).
usage: python3 tools/prof_binom.py gpurun_out/prof_<tag> [L cols]"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main(d, t=128, n=8192):
    """t = L (positions per piece), n = columns (pieces x 2 x dealers)."""
    rows = [r for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv")))
            if "binom" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ded = os.environ.get("DKG_PROF_BINOM_COMPLETE") is None  # the dedicated items (default schedule)
    cost = {m: bench.binom_item_valu(m, bench.SLOTS, ded) for m in range(1, t)}
    seg = rows[:t - 1]
    tot = totw = 0
    for i, r in enumerate(seg):
        rr = i + 1
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        w = sum(cost[m] for m in range(1, rr + 1)) * n
        tot += dur
        totw += w
        if rr in (1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 120, 127, 128, 192, 255, 256, 257, 300, 384, 448, 500, 511):
            print(f"r={rr:4d} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']} dur={dur / 1e3:8.1f}us "
                  f"eff={w / (dur * 1e-9) / bench.INT32_PEAK * 100:5.1f}%")
    print("total %.1f ms eff %.1f%%" % (tot / 1e6, totw / (tot * 1e-9) / bench.INT32_PEAK * 100))
    gaps = sum(int(seg[i + 1]["Start_Timestamp"]) - int(seg[i]["End_Timestamp"]) for i in range(len(seg) - 1))
    print("gaps between launches %.2f ms" % (gaps / 1e6))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], *(int(x) for x in a[1:]))
