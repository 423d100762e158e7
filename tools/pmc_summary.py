"""Summarise rocprofv3 CSV output of tools/profile.sh per kernel (sums over dispatches).

usage: python3 tools/pmc_summary.py gpurun_out/prof_<tag> [--traffic profiles/pmc_traffic/<tag>.json
       --n N --t T --split U --split-len L [--batch B] [--mode full]]
Prints kernel-trace stats (calls, total/avg ms) and, per kernel, the SQ issue/wait split,
VALU instructions (wave-level x 64 lanes) and HBM-side bytes: FETCH_SIZE doubled (gfx950 counts
half the bytes of wide coalesced reads, MI355X_MICROARCH.md "HBM") and WRITE_SIZE, both in KB.
With --traffic (and the profiled workload's key) it also writes the per-launch HBM bytes of the
pipeline kernels, which bench.py reports as roofline.traffic for a line of the same workload.
"""
import csv
import json
import os
import re
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


def eff_clock(path):
    """Per kernel: (sum of GRBM_GUI_ACTIVE, sum of dispatch durations in ns) over its dispatches of the
    pass at `path`.  GRBM_GUI_ACTIVE / 8 / duration is the clock the chip held during the kernel
    (MI355X_MICROARCH.md "DVFS give-back": rocprofv3 sums the counter over the 8 XCDs; it reads high
    on dispatches shorter than ~0.3 ms and is within 3 % of the in-kernel clock from 10 ms on)."""
    out = defaultdict(lambda: [0.0, 0.0])
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            e = out[short(row["Kernel_Name"])]
            e[0] += float(row["Counter_Value"])
            e[1] += int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return out


def main(d):
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    print(f"{'kernel':24s} {'calls':>6s} {'total ms':>10s} {'avg us':>10s}")
    with open(stats) as f:
        for row in csv.DictReader(f):
            print(f"{short(row['Name']):24s} {int(row['Calls']):6d} {float(row['TotalDurationNs']) / 1e6:10.3f} "
                  f"{float(row['AverageNs']) / 1e3:10.1f}")
    clk = eff_clock(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    if clk:
        print()
        print("effective clock under load (pmc_fetch pass: GRBM_GUI_ACTIVE / 8 / dispatch time), kernels >= 1 ms:")
        for k, (g, ns) in sorted(clk.items(), key=lambda x: -x[1][1]):
            if ns >= 1e6:
                print(f"{k:40s} {g / 8 / ns * 1e3:7.0f} MHz over {ns / 1e6:9.3f} ms")
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
    va, vcalls = load_counters(os.path.join(d, "pmc_valu", "run_counter_collection.csv"))
    if va:
        print()
        print("VALU unit (pmc_valu): cyc/instr = SQ_THREAD_CYCLES_VALU / (64 x SQ_INSTS_VALU), the SIMD cycles a")
        print("wave64 VALU instruction occupies (2 for a full-rate one on a 32-lane SIMD); slots/instr = cyc/instr / 2,")
        print("the roofline's issue-slot unit (bench.py: half-rate instructions count 2)")
        print(f"{'kernel':24s} {'disp':>5s} {'INSTS_VALU x64':>15s} {'THREAD_CYC':>12s} {'cyc/instr':>9s} {'slots/instr':>11s} "
              f"{'INT64/VALU':>10s} {'INT32/VALU':>10s} {'ACTIVE_VALU/INSTS':>17s} {'VALU2/ACTIVE':>12s}")
        for k in sorted(va, key=lambda k: -va[k].get("SQ_THREAD_CYCLES_VALU", 0)):
            c = va[k]
            ins = c.get("SQ_INSTS_VALU", 0) or 1
            print(f"{k:24s} {len(vcalls[k]):5d} {ins * 64:15.4g} {c.get('SQ_THREAD_CYCLES_VALU', 0):12.4g} "
                  f"{c.get('SQ_THREAD_CYCLES_VALU', 0) / (64 * ins):9.3f} "
                  f"{c.get('SQ_THREAD_CYCLES_VALU', 0) / (128 * ins):11.3f} "
                  f"{c.get('SQ_INSTS_VALU_INT64', 0) / ins:10.3f} {c.get('SQ_INSTS_VALU_INT32', 0) / ins:10.3f} "
                  f"{c.get('SQ_ACTIVE_INST_VALU', 0) / ins:17.3f} "
                  f"{c.get('SQ_ACTIVE_INST_VALU2', 0) / (c.get('SQ_ACTIVE_INST_VALU', 0) or 1):12.4f}")


def phase(name, ded_binomial=False):
    """Pipeline phase of a kernel-trace name (template arguments as rocprofv3 prints them): the
    dedicated stepping (k_stepping<MAXBS, true, PARTS>) and its complete-formula redo launches
    (<MAXBS, false, ..>: near-empty when no workgroup was marked, kept apart so that they do not
    halve the per-launch average), the recombination, the normalisation, the binomial (per step or
    per wave; with ded_binomial -- the run had a dedicated k_binom_wave<.., .., true> / k_binom_step<true>
    -- the complete variants are its redo launches, "binomial_redo"), the check and full mode's
    hybrid kernels."""
    m = re.match(r"(?:void )?k_binom_(?:wave<\w+, \w+, (true|false)>|step<(true|false)>)", name)
    if m and ded_binomial:
        return "binomial" if "true" in (m.group(1), m.group(2)) else "binomial_redo"
    if name == "k_binom_step" or re.match(r"(void )?k_binom_(wave|step)<", name):
        return "binomial"
    m = re.match(r"void k_stepping<\d+(?:, (true|false))?", name)
    if m:
        return "stepping_redo" if m.group(1) == "false" else "stepping"
    if re.match(r"void k_combine(_aff|_short)?<", name):
        return "combine"
    if re.match(r"(void )?k_check_both(<\d>)?$", name):  # <0> fused; <1> / <2> the g and h comb passes
        return "check"
    return {"k_affine_pieces": "affine", "k_check_both": "check", "k_check": "check", "k_commit": "commit",
            "k_enc_mul": "enc_mul", "k_dec_mul_w4": "dec_mul", "k_sym_xor": "sym"}.get(name)


def write_traffic(d, out, key):
    """Per-launch HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, counted in separate --pmc passes) of the
    pipeline kernels, summed over every dispatch the profiled run made, under the workload `key`
    (n, t, split, split_len, batch, mode) bench.py matches its line against."""
    fe, fcalls = load_counters(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    wr, wcalls = load_counters(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    kern = {}
    ded = any(re.match(r"(?:void )?k_binom_(?:wave<\w+, \w+, true>|step<true>)", k) for k in fe)
    for k in fe:
        ph = phase(k, ded)
        if ph is None or k not in wr:
            continue
        e = kern.setdefault(ph, {"fetch_bytes_x2": 0.0, "write_bytes": 0.0, "fetch_launches": 0, "write_launches": 0})
        e["fetch_bytes_x2"] += 2 * fe[k].get("FETCH_SIZE", 0) * 1024  # FETCH_SIZE and WRITE_SIZE are in KiB
        e["write_bytes"] += wr[k].get("WRITE_SIZE", 0) * 1024
        e["fetch_launches"] += len(fcalls[k])
        e["write_launches"] += len(wcalls[k])
    for e in kern.values():
        e["bytes_per_launch"] = (e["fetch_bytes_x2"] / max(e["fetch_launches"], 1)
                                 + e["write_bytes"] / max(e["write_launches"], 1))
    # the share of 64-bit VALU instructions (all half rate: the 64-bit mads and shifts) per phase, from
    # the pmc_valu pass: slots >= instructions x (1 + share), the counters' own lower bound on the
    # roofline's issue-slot unit (bench.py reports it beside frac and instr_frac)
    va, _ = load_counters(os.path.join(d, "pmc_valu", "run_counter_collection.csv"))
    agg = {}
    for k, c in va.items():
        ph = phase(k)
        if ph in kern:
            a = agg.setdefault(ph, [0.0, 0.0])
            a[0] += c.get("SQ_INSTS_VALU", 0)
            a[1] += c.get("SQ_INSTS_VALU_INT64", 0)
    for ph, (ins, i64) in agg.items():
        if ins:
            kern[ph]["valu_int64_share"] = i64 / ins
    # the clock each phase ran at in the profiled pass (GRBM_GUI_ACTIVE / 8 / time)
    # (only where the phase's dispatches average >= 1 ms: the counter reads high on short ones, so the
    # per-step binomial's ~0.15-ms launches get no figure)
    ck = {}
    for k, (g, ns) in eff_clock(os.path.join(d, "pmc_fetch", "run_counter_collection.csv")).items():
        ph = phase(k, ded)
        if ph in kern:
            a = ck.setdefault(ph, [0.0, 0.0])
            a[0] += g
            a[1] += ns
    for ph, (g, ns) in ck.items():
        if ns and ns / max(kern[ph]["fetch_launches"], 1) >= 1e6:
            kern[ph]["effective_clock_mhz"] = g / 8 / ns * 1e3
    doc = {"source": f"rocprofv3 --pmc FETCH_SIZE (doubled, MI355X_MICROARCH.md HBM) and --pmc WRITE_SIZE, "
                     f"separate passes of tools/profile.sh ({os.path.basename(os.path.normpath(d))})",
           "key": key, "kernels": kern}
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--traffic", help="write the per-launch traffic file here (needs --n --t --split)")
    ap.add_argument("--n", type=int)
    ap.add_argument("--t", type=int)
    ap.add_argument("--split", type=int)
    ap.add_argument("--split-len", type=int)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--mode", default="plain")
    a = ap.parse_args()
    main(a.dir)
    if a.traffic:
        write_traffic(a.dir, a.traffic, {"n": a.n, "t": a.t, "split": a.split, "split_len": a.split_len,
                                         "batch": a.batch, "mode": a.mode})
