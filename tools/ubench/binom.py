"""Prices tools/ubench/binom's output: the closed-form VALU issue slots of one Horner step of the
headline tables (8192 columns, positions m = 1..r) in each variant, over the measured launch time,
as a fraction of the slot peak (bench.py units).
usage: python3 tools/ubench/binom.py gpurun_out/<tag>/binom.log"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

V = bench.SLOTS
COLS = 8192


def item(m, part):
    """Slots of one dedicated item e_m = m (e_{m-1} + e_m): 'full' (first addition + m-chain,
    bench.binom_item_valu) or 'chain' (the m-chain alone, as the chain variant runs it)."""
    c = bench.binom_item_valu(m)
    if part == "chain":
        c -= V["ge_to_cached_ded"] + V["ge_add_ded"] + V["fe_tight_zero"]
    return c


def main(path):
    for line in open(path):
        mt = re.match(r"(\w+) r=(\d+) us=([\d.]+)", line)
        if not mt:
            continue
        var, r, us = mt.group(1), int(mt.group(2)), float(mt.group(3))
        work = COLS * sum(item(m, "chain" if var == "chain" else "full") for m in range(1, r + 1))
        print(f"{var:8s} r={r:4d} {us:8.1f} us  frac {work / (us * 1e-6) / bench.INT32_PEAK:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
