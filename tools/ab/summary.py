#!/usr/bin/env python3
"""Summary of a tools/ab/ab.sh run: per variant, the JSON lines' ms_per_step (bench.py) or ms_wall
(tools/shard_time.py, per ws) over the rounds (min / median)."""
import collections
import glob
import json
import os
import statistics
import sys


def main(d):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "*.out"))):
        name = os.path.basename(f).rsplit(".", 2)[0]
        for line in open(f):
            line = line.strip()
            if not line.startswith("{"):
                continue
            j = json.loads(line)
            if "ms_per_step" in j:
                vals[(name, "step")].append(j["ms_per_step"])
            elif "ms_wall" in j:
                vals[(name, f"ws{j['ws']}")].append(j["ms_wall"])
    for (name, key), v in sorted(vals.items()):
        print(f"{name:24s} {key:6s} min {min(v):9.3f}  median {statistics.median(v):9.3f}  n={len(v)}")


if __name__ == "__main__":
    main(sys.argv[1])
