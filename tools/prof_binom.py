"""Per-launch efficiency of the binomial step kernel from a rocprofv3 kernel-trace database."""
import glob
import sqlite3
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
t = int(sys.argv[2]) if len(sys.argv) > 2 else 511
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
c = sqlite3.connect(db)
rows = c.execute("select grid_x, grid_y, workgroup_x, duration, start from kernels where name like '%binom%' "
                 "order by start").fetchall()
V = bench.VALU
cost = {}
for m in range(1, t + 1):
    ds = bench._naf(m)
    cc = V["ge_to_cached"] + V["ge_add"]
    if len(ds) > 1:
        cc += V["ge_to_cached"]
        for i in range(len(ds) - 2, -1, -1):
            nz = ds[i] != 0
            cc += V["ge_dbl_t"] if (nz or i == 0) else V["ge_dbl_not"]
            if nz:
                cc += V["ge_add_signed"]
    cost[m] = cc
seg = rows[:t]
for r in [1, 2, 4, 8, 16, 32, 64, 128, 192, 256, 320, 384, 448, 511]:
    if r > len(seg):
        break
    gx, gy, wx, dur, st = seg[r - 1]
    work = sum(cost[m] for m in range(1, r + 1)) * n
    print(f"r={r:4d} grid={gx}x{gy} dur={dur / 1e3:8.1f}us  eff={work / (dur * 1e-9) / bench.INT32_PEAK * 100:5.1f}%")
tot = sum(r[3] for r in seg)
gaps = sum(seg[i + 1][4] - (seg[i][4] + seg[i][3]) for i in range(len(seg) - 1))
print("total binom kernel time %.1f ms, gaps %.1f ms" % (tot / 1e6, gaps / 1e6))
