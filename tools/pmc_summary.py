"""Summarise rocprofv3 CSV output of tools/profile.sh per kernel (sums over dispatches).

usage: python3 tools/pmc_summary.py gpurun_out/prof_<tag>
Prints kernel-trace stats (calls, total/avg ms) and, per kernel, the SQ issue/wait split,
VALU instructions (wave-level x 64 lanes) and HBM-side bytes: FETCH_SIZE doubled (gfx950 counts
half the bytes of wide coalesced reads, MI355X_MICROARCH.md "HBM") and WRITE_SIZE, both in KB.
"""
import csv
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("dkgk::", "")


def load_counters(path):
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    if not os.path.exists(path):
        return agg, calls
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
            calls[k].add(row["Dispatch_Id"])
    return agg, calls


def main(d):
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    print(f"{'kernel':24s} {'calls':>6s} {'total ms':>10s} {'avg us':>10s}")
    with open(stats) as f:
        for row in csv.DictReader(f):
            print(f"{short(row['Name']):24s} {int(row['Calls']):6d} {float(row['TotalDurationNs']) / 1e6:10.3f} "
                  f"{float(row['AverageNs']) / 1e3:10.1f}")
    sq, calls = load_counters(os.path.join(d, "pmc_sq", "run_counter_collection.csv"))
    fe, _ = load_counters(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    wr, _ = load_counters(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    print()
    print(f"{'kernel':24s} {'disp':>5s} {'VALU lane-instr':>16s} {'active%':>8s} {'wait%':>7s} {'waitinst%':>9s} "
          f"{'valu/active':>11s} {'fetch MB x2':>12s} {'write MB':>10s}")
    for k in sorted(sq, key=lambda k: -sq[k].get("SQ_WAVE_CYCLES", 0)):
        c = sq[k]
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"{k:24s} {len(calls[k]):5d} {c.get('SQ_INSTS_VALU', 0) * 64:16.4g} "
              f"{100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc:8.1f} {100 * c.get('SQ_WAIT_ANY', 0) / wc:7.1f} "
              f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:9.1f} "
              f"{c.get('SQ_ACTIVE_INST_VALU', 0) / (c.get('SQ_ACTIVE_INST_ANY', 0) or 1):11.2f} "
              f"{2 * fe[k].get('FETCH_SIZE', 0) / 1e3:12.1f} {wr[k].get('WRITE_SIZE', 0) / 1e3:10.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
