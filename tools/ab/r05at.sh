#!/bin/bash
# Round 5, final tree: config 5's bench line (its batch path is unchanged since r05ae; re-measured so
# that every final line comes from the final tree) with its CPU baseline and the committed traffic file.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05at
mkdir -p $O
timeout -k 10 400 python bench.py --config B5 --steps 5 --warmup 1 > $O/bench_B5.json 2> $O/bench_B5.err || { echo BENCH B5 FAILED; tail -20 $O/bench_B5.err; exit 1; }
cut -c1-200 $O/bench_B5.json
echo ALL DONE
