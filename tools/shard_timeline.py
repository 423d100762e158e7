"""Timeline of the last call in a rocprofv3 kernel trace (run_kernel_trace.csv): where the device
time of one dealer-shard ceremony goes, kernel by kernel, and how long the device sat idle.

A "call" is a maximal run of launches without an idle gap longer than --gap-ms; the last one that
holds a kernel named like --with (default k_stepping) is analysed.  Prints per-kernel-name busy time (union of
overlapping launches counted once per name) and the idle time between launches within the call.
usage: python tools/shard_timeline.py <run_kernel_trace.csv> [--gap-ms 2.0] [--top 25]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-ms", type=float, default=2.0, help="an idle gap longer than this separates calls")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--with", dest="with_", default="k_stepping", help="the last call holding a kernel of this name")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # calls = maximal runs of launches without an idle gap > gap-ms
    calls, cur, end = [], [], None
    for s, e, k in rows:
        if end is not None and s - end > a.gap_ms * 1e6:
            calls.append(cur)
            cur = []
        cur.append((s, e, k))
        end = e if end is None else max(end, e)
    calls.append(cur)
    call = [c for c in calls if any(a.with_ in k for _, _, k in c)][-1]
    t0, t1 = call[0][0], max(e for _, e, _ in call)
    busy = collections.defaultdict(float)
    count = collections.Counter()
    for s, e, k in call:
        busy[k.split("(")[0][:60]] += (e - s) / 1e6
        count[k.split("(")[0][:60]] += 1
    # idle: device time covered by no launch
    idle, cover_end = 0.0, t0
    for s, e, _ in call:
        if s > cover_end:
            idle += (s - cover_end) / 1e6
        cover_end = max(cover_end, e)
    print(f"{len(calls)} calls in the trace; the last: {len(call)} launches over {(t1 - t0) / 1e6:.3f} ms, "
          f"device idle between launches {idle:.3f} ms")
    for k, v in sorted(busy.items(), key=lambda x: -x[1])[:a.top]:
        print(f"  {k:60s} {count[k]:5d} launches {v:9.3f} ms")


if __name__ == "__main__":
    main()
